"""Helpers to load the committed golden vectors and the oracle library
(test infrastructure only)."""
import ctypes
import gzip
import json
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE_SO = os.path.join(REPO, "oracle", "_build", "liboracle.so")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def edge_cases():
    with open(os.path.join(GOLDEN, "edge_cases.json")) as f:
        return json.load(f)


def gz(name):
    with gzip.open(os.path.join(GOLDEN, name), "rb") as f:
        return f.read()


_oracle = None


def oracle():
    """ctypes handle to the C restatement (built by `make -C oracle`)."""
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"),
                            os.path.join(REPO, "oracle", "_build", "liboracle.so")], check=True)
        lib = ctypes.CDLL(ORACLE_SO)
        u8p, szp = ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t)
        lib.vcfo_encode_line.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, szp]
        lib.vcfo_compress.argtypes = [u8p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, szp,
                                      ctypes.POINTER(ctypes.c_int64)]
        lib.vcfo_decompress.argtypes = [u8p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, szp]
        u64 = ctypes.c_uint64
        lib.vcfo_parse_query.argtypes = [u8p, ctypes.c_size_t, szp, ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(u64), ctypes.POINTER(u64)]
        lib.vcfo_query.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, ctypes.c_int, u64, u64,
                                   ctypes.c_void_p, ctypes.c_size_t, szp]
        lib.vcfo_sparsify.argtypes = [u8p, ctypes.c_size_t, ctypes.c_char_p]
        lib.vcfo_sparse_offset.restype = ctypes.c_uint64
        lib.vcfo_sparse_offset.argtypes = [ctypes.c_uint64]
        lib.vcfo_encode_bound.restype = ctypes.c_size_t
        lib.vcfo_encode_bound.argtypes = [ctypes.c_size_t]
        _oracle = lib
    return _oracle


def oracle_encode_line(line, add_newline=True):
    lib = oracle()
    cap = lib.vcfo_encode_bound(len(line))
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    st = lib.vcfo_encode_line(line, len(line), int(add_newline), buf, cap, ctypes.byref(n))
    return st, buf.raw[:n.value]


def oracle_hash64(rec):
    """vcfo_hash64: the record digest vcfc_record_hash_device computes."""
    lib = oracle()
    lib.vcfo_hash64.restype = ctypes.c_uint64
    lib.vcfo_hash64.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    return lib.vcfo_hash64(rec, len(rec))


def oracle_encode_rows_hash(buf, line_off, line_len, threads=8):
    """Threaded oracle encode of rows buf[line_off[i] .. + line_len[i]):
    (status int32[n], record size uint32[n], digest uint64[n]).  `buf` is a
    numpy uint8 array (or bytes)."""
    import numpy as np
    lib = oracle()
    vp = ctypes.c_void_p
    lib.vcfo_encode_rows_hash.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_int, vp, vp, vp]
    b = np.frombuffer(buf, dtype=np.uint8) if isinstance(buf, (bytes, bytearray)) else buf
    off = np.ascontiguousarray(line_off, dtype=np.uint64)
    ln = np.ascontiguousarray(line_len, dtype=np.uint32)
    n = len(off)
    st = np.zeros(n, dtype=np.int32)
    size = np.zeros(n, dtype=np.uint32)
    h = np.zeros(n, dtype=np.uint64)
    assert lib.vcfo_encode_rows_hash(b.ctypes.data, off.ctypes.data, ln.ctypes.data, n, threads, h.ctypes.data,
                                     size.ctypes.data, st.ctypes.data) == 0
    return st, size, h


def oracle_compress(data):
    lib = oracle()
    cap = len(data) * 2 + 1024
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    err = ctypes.c_int64(0)
    st = lib.vcfo_compress(data, len(data), buf, cap, ctypes.byref(n), ctypes.byref(err))
    return st, buf.raw[:n.value], err.value


def oracle_decompress(data, cap=None):
    lib = oracle()
    cap = cap or len(data) * 8 + 1024
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    st = lib.vcfo_decompress(data, len(data), buf, cap, ctypes.byref(n))
    return st, buf.raw[:n.value]


def oracle_parse_query(q):
    """parse_coordinate_string: None on failure, else (ref, has_range, start, end)."""
    lib = oracle()
    rl, hr = ctypes.c_size_t(0), ctypes.c_int(0)
    a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
    if lib.vcfo_parse_query(q, len(q), ctypes.byref(rl), ctypes.byref(hr), ctypes.byref(a), ctypes.byref(b)) != 0:
        return None
    return q[:rl.value], bool(hr.value), a.value, b.value


def oracle_query(data, q, cap=None):
    """query_compressed_file over bytes: (status, matching lines)."""
    lib = oracle()
    pq = oracle_parse_query(q)
    assert pq is not None
    ref, hr, a, b = pq
    cap = cap or len(data) * 600 + 4096
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    st = lib.vcfo_query(data, len(data), ref, len(ref), int(hr), a, b, buf, cap, ctypes.byref(n))
    return st, buf.raw[:n.value]


def query_cases():
    """(case dict, file bytes) for tests/golden/query_cases.json."""
    d = json.load(open(os.path.join(GOLDEN, "query_cases.json")))
    files = {k: bytes.fromhex(v) for k, v in d["inline_files"].items()}
    for k, (src, frac) in d["truncated_from"].items():
        full = gz(src)
        files[k] = full[:len(full) * 2 // 3]
    for c in d["cases"]:
        f = c["file"]
        yield c, files[f] if f in files else gz(f)


def oracle_sparse_query(path, q, cap=1 << 26):
    """query_sparse_file_fd over a sparse file: (status, stdout bytes)."""
    lib = oracle()
    if not hasattr(lib, "_sq"):
        lib.vcfo_sparse_query.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_size_t)]
        lib._sq = True
    ref, hr, a, b = oracle_parse_query(q)
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    st = lib.vcfo_sparse_query(path.encode(), ref, len(ref), int(hr), a, b, buf, cap, ctypes.byref(n))
    return st, buf.raw[:n.value]


def oracle_sparsify(vcfc, path):
    st = oracle().vcfo_sparsify(vcfc, len(vcfc), path.encode())
    assert st == 0, st


def _header_end(v):
    p = 0
    while v[p:p + 1] == b"#":
        p = v.index(b"\n", p) + 1
    return p


def _samples_delta(v, delta):
    h = _header_end(v)
    lines = v[:h].split(b"\n")[:-1]
    cols = lines[-1].split(b"\t")
    cols = cols + [b"EXTRA"] * delta if delta > 0 else cols[:len(cols) + delta]
    lines[-1] = b"\t".join(cols)
    return b"\n".join(lines) + b"\n" + v[h:]


def sparse_query_cases():
    """json of tests/golden/sparse_query_cases.json."""
    return json.load(open(os.path.join(GOLDEN, "sparse_query_cases.json")))


def build_sparse_file(d, name, path, sparsify):
    """Recreate sparse file `name` of the sparse-query goldens at `path`:
    sparsify(vcfc_bytes, path) (this build's or the oracle's), then the
    recorded patches and truncation."""
    spec = d["files"][name]
    base = d["bases"][spec["base"]]
    src = base["vcfc"]
    if src.startswith("inline:"):
        v = dict((k, bytes.fromhex(x)) for k, x in json.load(open(os.path.join(GOLDEN, "query_cases.json")))
                 ["inline_files"].items())[src[7:]]
    else:
        v = gz(src)
    if base["samples_delta"]:
        v = _samples_delta(v, base["samples_delta"])
    sparsify(v, path)
    with open(path, "r+b") as f:
        for off, hx in spec["patches"]:
            f.seek(off)
            f.write(bytes.fromhex(hx))
        if spec["truncate"] is not None:
            f.truncate(spec["truncate"])


def check_sparse_case(c, st, out):
    """A result against a golden case: exact stdout when the reference exits
    0; where it aborts (uncaught throw: rc -6/134), the reference's stdout is
    the flushed prefix of the lines before the throw, so ours must extend it
    and report VCFC_E_FORMAT (8)."""
    import hashlib
    if c["rc"] == 0:
        return st == 0 and len(out) == c["stdout_len"] and hashlib.sha256(out).hexdigest() == c["stdout_sha256"]
    return st == 8 and len(out) >= c["stdout_len"] and \
        hashlib.sha256(out[:c["stdout_len"]]).hexdigest() == c["stdout_sha256"]
