"""TEST INFRASTRUCTURE ONLY: ctypes binding of the fiber-emulated build of the
product kernels (tests/simt_emu) + helpers to index VCF data lines."""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU_SO = os.path.join(REPO, "tests", "simt_emu", "_build", "libvcfc_emu.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        import fcntl
        os.makedirs(os.path.dirname(EMU_SO), exist_ok=True)
        with open(EMU_SO + ".lock", "w") as lk:   # one build at a time (pytest -n workers)
            fcntl.flock(lk, fcntl.LOCK_EX)
            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "simt_emu")], check=True)
        L = ctypes.CDLL(EMU_SO)
        vp = ctypes.c_void_p
        L.emu_encode_rows.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint64, vp,
                                      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint32)]
        L.emu_last_deferred.restype = ctypes.c_uint32
        L.emu_last_mispredict.restype = ctypes.c_uint32
        L.emu_sparse_plan.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_uint64, vp, vp, vp]
        L.emu_decompress.argtypes = [ctypes.c_char_p, ctypes.c_uint64, vp, ctypes.c_uint64,
                                     ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
        u64 = ctypes.c_uint64
        L.emu_query.argtypes = [ctypes.c_char_p, u64, ctypes.c_char_p, u64, ctypes.c_int, u64, u64, vp, u64,
                                ctypes.POINTER(u64), u64]
        L.emu_sparse_query.argtypes = [ctypes.c_char_p, ctypes.c_char_p, u64, ctypes.c_int, u64, u64, ctypes.c_int]
        L.emu_compress.argtypes = [ctypes.c_char_p, u64, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_int64),
                                   u64, ctypes.c_int, u64]
        L.emu_record_hash.argtypes = [vp, vp, u64, vp]
        L.emu_compress_device.argtypes = [ctypes.c_char_p, u64, vp, u64, ctypes.POINTER(u64),
                                          ctypes.POINTER(ctypes.c_int64), u64, u64, ctypes.c_int,
                                          ctypes.POINTER(u64)]
        L.emu_line_index.argtypes = [ctypes.c_char_p, u64, ctypes.c_uint32, vp, vp, u64, vp, u64]
        L.emu_synth.argtypes = [vp, vp, u64, vp, vp, vp, ctypes.c_uint32, ctypes.c_int, u64, u64]
        _lib = L
    return _lib


def emu_record_hash(recs, rec_off):
    """Per-record digests of `recs` (bytes) at rec_off (n + 1) on the emulator."""
    n = len(rec_off) - 1
    out = np.zeros(max(n, 1), dtype=np.uint64)
    src = np.frombuffer(recs + b"\0" * 16, dtype=np.uint8)
    ro = np.ascontiguousarray(rec_off, dtype=np.uint64)
    st = lib().emu_record_hash(src.ctypes.data, ro.ctypes.data, n, out.ctypes.data)
    assert st == 0
    return out[:n]


def data_lines(vcf):
    """(buf, line_off, line_len) of the data lines of a VCF buffer, following
    compress()'s getline loop (reference src/compress.cpp:218-253): empty
    lines and '#' lines are not data lines."""
    offs, lens = [], []
    p, n = 0, len(vcf)
    while p < n:
        e = vcf.find(b"\n", p)
        e = n if e < 0 else e
        if e > p and vcf[p] != 0x23:
            offs.append(p)
            lens.append(e - p)
        p = e + 1
    return vcf, np.array(offs, dtype=np.uint64), np.array(lens, dtype=np.uint32)


LAST_RETRIES = [0]


def last_deferred():
    """Rows the last emu_encode call deferred (sized by k_encode_var, written
    to out by k_encode_defer)."""
    return int(lib().emu_last_deferred())


def last_mispredict():
    """Whether the last emu_encode call's first deferred pass found a
    predicted record size wrong (the size scan, compaction and deferred
    writes then ran again on exact sizes)."""
    return int(lib().emu_last_mispredict())


def emu_encode(buf, line_off, line_len, cap=None):
    """Run the product encode pipeline on the emulator (output capacity
    `cap`, default the bound).  Returns (status, records bytes, rec_off
    array, err_word); the number of rows the fast kernel handed to the
    general kernel is left in LAST_RETRIES[0]."""
    n = len(line_off)
    full = int(sum(int(x) * 3 // 2 + 32 for x in line_len)) + 64
    cap = full if cap is None else cap
    out = np.zeros(max(cap, full), dtype=np.uint8)   # (bytes past cap must stay untouched)
    rec_off = np.zeros(n + 1, dtype=np.uint64)
    src = np.frombuffer(buf, dtype=np.uint8).copy()
    lo = np.ascontiguousarray(line_off, dtype=np.uint64)
    ll = np.ascontiguousarray(line_len, dtype=np.uint32)
    err = ctypes.c_uint64(0)
    sw = ctypes.c_uint64(0)
    rt = ctypes.c_uint32(0)
    st = lib().emu_encode_rows(src.ctypes.data, lo.ctypes.data, ll.ctypes.data, n, out.ctypes.data, cap,
                               rec_off.ctypes.data, ctypes.byref(err), ctypes.byref(sw), ctypes.byref(rt))
    LAST_RETRIES[0] = rt.value
    total = int(rec_off[n]) if n else 0
    if cap < full:
        assert not out[cap:].any(), "bytes written past out_cap"
    return st, out[:total].tobytes(), rec_off, err.value


def emu_sparse_plan(recs, rec_off, data_start):
    """Run k_sparse_plan on the emulator: (file_off, prefix16 bytes, status[2])."""
    n = len(rec_off) - 1
    src = np.frombuffer(recs, dtype=np.uint8).copy()
    ro = np.ascontiguousarray(rec_off, dtype=np.uint64)
    fo = np.zeros(max(n, 1), dtype=np.uint64)
    pf = np.zeros(16 * max(n, 1), dtype=np.uint8)
    stt = np.zeros(2, dtype=np.uint64)
    lib().emu_sparse_plan(src.ctypes.data, ro.ctypes.data, n, data_start, fo.ctypes.data, pf.ctypes.data,
                          stt.ctypes.data)
    return fo[:n], pf[:16 * n].tobytes(), stt


def emu_decompress(data, out_batch=1 << 16, cap=None):
    """Run the product decode driver + kernels on the emulator: (status, bytes)."""
    cap = cap or len(data) * 600 + 4096
    out = np.zeros(cap, dtype=np.uint8)
    n = ctypes.c_uint64(0)
    st = lib().emu_decompress(data, len(data), out.ctypes.data, cap, ctypes.byref(n), out_batch)
    return st, out[:n.value].tobytes()


def emu_query(data, ref, has_range, start, end, out_batch=1 << 16, cap=None):
    """Run the product query driver + kernels on the emulator: (status, bytes)."""
    cap = cap or len(data) * 600 + 4096
    out = np.zeros(cap, dtype=np.uint8)
    n = ctypes.c_uint64(0)
    st = lib().emu_query(data, len(data), ref, len(ref), int(has_range), start, end, out.ctypes.data, cap,
                         ctypes.byref(n), out_batch)
    return st, out[:n.value].tobytes()


def emu_sparse_query(path, ref, has_range, start, end):
    """The product sparse-query driver + kernels on the emulator: (status, bytes)."""
    import tempfile
    with tempfile.TemporaryFile() as f:
        st = lib().emu_sparse_query(path.encode(), ref, len(ref), int(has_range), start, end, f.fileno())
        f.seek(0)
        return st, f.read()


def emu_compress(vcf, chunk=4096, read_threads=2, cap=None, max_chunk=0):
    """compress() through the product ingest pipeline on the emulator:
    (status, bytes, err_line)."""
    cap = cap or 2 * len(vcf) + 4096
    out = np.zeros(cap, dtype=np.uint8)
    n = ctypes.c_uint64(0)
    el = ctypes.c_int64(-1)
    st = lib().emu_compress(vcf, len(vcf), out.ctypes.data, cap, ctypes.byref(n), ctypes.byref(el), chunk,
                            read_threads, max_chunk)
    return st, out[:n.value].tobytes(), el.value


def emu_compress_device(vcf, chunk=4096, cap=None, max_chunk=0, hop=True, redo=None):
    """compress() of device-resident bytes (vcfc_ing::compress_device) on the
    emulator: (status, bytes, err_line).  hop: the hop line index when the
    header gives S (True; "learn" / "nolearn" force its learned candidates on
    or off); redo (a list): gets the count of chunks indexed again."""
    cap = cap or 2 * len(vcf) + 4096
    out = np.zeros(cap, dtype=np.uint8)
    n = ctypes.c_uint64(0)
    el = ctypes.c_int64(-1)
    r = ctypes.c_uint64(0)
    st = lib().emu_compress_device(vcf, len(vcf), out.ctypes.data, cap, ctypes.byref(n), ctypes.byref(el), chunk,
                                   max_chunk, {"learn": 2, "nolearn": 3}.get(hop, 1 if hop else 0), ctypes.byref(r))
    if redo is not None:
        redo.append(r.value)
    return st, out[:n.value].tobytes(), el.value


def emu_hop_read(reset=True):
    """Bytes the hop line index's walkers loaded since the last reset (the
    emulator's VCFC_DIAG_HOP_READ counter)."""
    L = lib()
    L.emu_hop_read.restype = ctypes.c_ulonglong
    L.emu_hop_read.argtypes = [ctypes.c_int]
    return int(L.emu_hop_read(1 if reset else 0))


def emu_line_index(vcf, S_hint=0, hop_walkers=0, learn=True, len_hint=0):
    """The GPU line index of vcf (ending in '\n') on the emulator: (counts
    [lines, data lines, pass lines, long], data line offsets, lengths).
    hop_walkers: walkers of the hop index (0: the product's count); learn:
    the walkers with learned candidates (TRY / LEARN), else the GUESS ones
    (compress_device's choice for chr22-shaped files); len_hint: the GUESS
    walkers' first line length (compress_device: the first data line's)."""
    cap = vcf.count(b"\n") + 1
    off = np.zeros(cap, dtype=np.uint64)
    ln = np.zeros(cap, dtype=np.uint32)
    cnt = np.zeros(4, dtype=np.uint64)
    L = lib()
    L.emu_line_index.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32]
    st = L.emu_line_index(vcf, len(vcf), S_hint, off.ctypes.data, ln.ctypes.data, cap, cnt.ctypes.data, hop_walkers,
                          1 if learn else 0, len_hint)
    assert st == 0
    k = int(cnt[1])
    return [int(c) for c in cnt], off[:k].tolist(), ln[:k].tolist()


def emu_synth_rows(n, samples, law, seed, row0=0, rows_of=None):
    """vcf-compression_amd/workload.py's synthetic rows generated by the
    product generator kernel on the emulator: (buf, line_off, line_len).
    rows_of = (n_total, lo): rows [lo, lo + n) of the n_total-row batch
    (workload.DeviceRows' slices)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "vcf-compression_amd"))
    import workload
    if rows_of is None:
        blob, poff, af, _, gt_len = workload.prefixes(n, law, seed, row0, samples)
        row_base = 0
    else:
        blob, poff, af, _, gt_len = workload.slice_prefixes(rows_of[0], rows_of[1], rows_of[1] + n, law, seed,
                                                             samples)
        row_base = rows_of[1]
    line_off, line_len, total = workload.layout(poff, samples, gt_len)
    buf = np.zeros(total + 64, dtype=np.uint8)
    pre = np.frombuffer(blob, dtype=np.uint8).copy()
    lo = np.ascontiguousarray(line_off, dtype=np.uint64)
    po = np.ascontiguousarray(poff, dtype=np.uint64)
    afp = af.ctypes.data if af is not None else None
    assert lib().emu_synth(buf.ctypes.data, lo.ctypes.data, n, pre.ctypes.data, po.ctypes.data, afp, samples, law,
                           seed, row_base) == 0
    return buf[:total], lo, np.ascontiguousarray(line_len, dtype=np.uint32)
