"""Python binding (ctypes) of libvcfc.so -- the C ABI in include/vcfc.h.

Mirrors the reference's operator interface for the encode path:
  compress_data_line(line, add_newline=True)   (reference src/compress.hpp:20-23)
  compress_file(in_path, out_path)             (reference src/compress.cpp:205-257)
  decompress / decompress_file                 (reference src/compress.cpp:1214-1257)
  parse_coordinate_string, query / query_file  (reference src/main.cpp:3777-4026)
Errors raise VcfValidationError / RuntimeError like the reference's exceptions
(src/utils.hpp:117-123, src/compress.cpp:9-11,231-234).

There is no CPU fallback: without a visible gfx950 GPU, Context() raises.
If PyTorch is used in the same process, import torch BEFORE loading this
module so both share one HIP runtime (libvcfc.so binds to whatever
libamdhip64.so is already loaded).
"""
import collections
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("VCFC_LIB") or os.path.join(ROOT, "build", "libvcfc.so")

OK, E_LT8COLS, E_8COLS, E_HEADER, E_NOSPACE, E_ARG, E_HIP, E_IO, E_FORMAT = range(9)
E_TOOLONG = 10   # a data line longer than MAX_LINE (include/vcfc.h VCFC_E_TOOLONG)
MAX_LINE = (1 << 29) - 64
NO_ERROR = (1 << 64) - 1

EXPORTS = [
    "vcfc_version", "vcfc_strerror", "vcfc_ctx_create", "vcfc_ctx_destroy",
    "vcfc_compress_data_line", "vcfc_encode_bound", "vcfc_encode_workspace_size",
    "vcfc_encode_rows_device", "vcfc_encode_rows", "vcfc_compress_file",
    "vcfc_compress_bound", "vcfc_compress_buffer", "vcfc_synth_rows_device", "vcfc_synth_rows_device_at",
    "vcfc_timer_create", "vcfc_timer_destroy", "vcfc_encode_rows_device_timed", "vcfc_timer_read",
    "vcfc_sparse_offset", "vcfc_sparsify_file", "vcfc_sparse_plan_device",
    "vcfc_decompress_buffer", "vcfc_decompress_file", "vcfc_decode_workspace_size",
    "vcfc_decode_records_device", "vcfc_parse_query", "vcfc_query_buffer", "vcfc_query_file",
    "vcfc_query_match_device", "vcfc_decode_selected_device", "vcfc_sparse_query_file",
    "vcfc_sparsify_shard", "vcfc_ctx_set_ingest_chunk", "vcfc_record_hash_device",
    "vcfc_compress_range", "vcfc_compress_device", "vcfc_compress_range_held", "vcfc_held_place",
    "vcfc_held_sizes", "vcfc_held_free", "vcfc_ctx_set_line_index", "vcfc_ctx_set_trace",
    "vcfc_ctx_set_deferred_records", "vcfc_encode_deferred_rows",
]
LINE_INDEX_HOP, LINE_INDEX_SCAN = 0, 1                       # include/vcfc.h VCFC_LINE_INDEX_*
TRACE_INGEST, TRACE_DEVICE, TRACE_SPARSE_QUERY = 1, 2, 4     # include/vcfc.h VCFC_TRACE_*


class VcfValidationError(RuntimeError):
    """Same meaning as the reference's VcfValidationError (src/utils.hpp:117-123)."""


class LengthError(RuntimeError):
    """The reference aborts with std::length_error on 8-column data lines."""


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libvcfc.so not built: run `make -C vcf-compression_amd` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, u32, i64 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64
    L.vcfc_version.restype = ctypes.c_char_p
    L.vcfc_strerror.restype = ctypes.c_char_p
    L.vcfc_strerror.argtypes = [ctypes.c_int]
    L.vcfc_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.vcfc_ctx_destroy.argtypes = [vp]
    L.vcfc_ctx_destroy.restype = None
    L.vcfc_ctx_set_ingest_chunk.argtypes = [vp, u64]
    # Exports added since round 3 are bound only when present: A/B runs load
    # older builds of the library (tools/ab.sh, VCFC_LIB); calling one that
    # the loaded build lacks raises a clear error (_need).  test_capi checks
    # that the current build exports every one of them.
    late = {"vcfc_ctx_set_line_index": [vp, ctypes.c_int], "vcfc_ctx_set_trace": [vp, ctypes.c_uint],
            "vcfc_ctx_set_deferred_records": [vp, ctypes.c_int],
            "vcfc_encode_deferred_rows": [vp, u64, u64, vp, ctypes.POINTER(u64)]}
    for name, args in late.items():
        if hasattr(L, name):
            getattr(L, name).argtypes = args
    L.vcfc_record_hash_device.argtypes = [vp, vp, u64, vp, vp]
    L.vcfc_compress_range.argtypes = [vp, ctypes.c_char_p, u64, u64, ctypes.c_int, u64, ctypes.POINTER(u64),
                                      ctypes.POINTER(i64), ctypes.POINTER(u64)]
    L.vcfc_compress_range_held.argtypes = [vp, ctypes.c_char_p, u64, u64, u64, ctypes.c_char_p, ctypes.POINTER(vp),
                                           ctypes.POINTER(u64), ctypes.POINTER(i64), ctypes.POINTER(u64)]
    L.vcfc_held_place.argtypes = [vp, ctypes.c_int, u64]
    L.vcfc_held_sizes.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    L.vcfc_held_sizes.restype = None
    L.vcfc_held_free.argtypes = [vp]
    L.vcfc_held_free.restype = None
    L.vcfc_compress_data_line.argtypes = [vp, ctypes.c_char_p, u64, ctypes.c_int, vp, u64, ctypes.POINTER(u64)]
    L.vcfc_encode_bound.restype = u64
    L.vcfc_encode_bound.argtypes = [u64, u64]
    L.vcfc_encode_workspace_size.restype = u64
    L.vcfc_encode_workspace_size.argtypes = [u64, u64]
    L.vcfc_encode_rows_device.argtypes = [vp, vp, vp, u64, u64, vp, u64, vp, vp, u64, vp, vp]
    L.vcfc_encode_rows.argtypes = [vp, vp, u64, vp, vp, u64, vp, u64, vp, ctypes.POINTER(i64)]
    L.vcfc_compress_file.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(i64)]
    L.vcfc_compress_bound.restype = u64
    L.vcfc_compress_bound.argtypes = [u64]
    L.vcfc_compress_buffer.argtypes = [vp, vp, u64, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(i64)]
    L.vcfc_compress_device.argtypes = [vp, vp, u64, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(i64)]
    L.vcfc_timer_create.argtypes = [ctypes.POINTER(vp)]
    L.vcfc_timer_destroy.argtypes = [vp]
    L.vcfc_timer_destroy.restype = None
    L.vcfc_encode_rows_device_timed.argtypes = [vp, vp, vp, u64, u64, vp, u64, vp, vp, u64, vp, vp, vp]
    L.vcfc_timer_read.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64)]
    L.vcfc_sparse_offset.restype = u64
    L.vcfc_sparse_offset.argtypes = [u64]
    L.vcfc_sparsify_file.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p]
    L.vcfc_sparsify_shard.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(u64)]
    L.vcfc_sparse_plan_device.argtypes = [vp, vp, u64, u64, vp, vp, vp, vp]
    L.vcfc_decompress_buffer.argtypes = [vp, vp, u64, vp, u64, ctypes.POINTER(u64)]
    L.vcfc_decompress_file.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p]
    L.vcfc_decode_workspace_size.restype = u64
    L.vcfc_decode_workspace_size.argtypes = [u64]
    L.vcfc_decode_records_device.argtypes = [vp, u64, vp, u64, u64, vp, u64, vp, vp, u64, vp, ctypes.c_int, vp]
    L.vcfc_synth_rows_device.argtypes = [vp, vp, u64, vp, vp, vp, u32, ctypes.c_int, u64, vp]
    L.vcfc_synth_rows_device_at.argtypes = [vp, vp, u64, vp, vp, vp, u32, ctypes.c_int, u64, u64, vp]
    pu64 = ctypes.POINTER(u64)
    L.vcfc_parse_query.argtypes = [ctypes.c_char_p, u64, pu64, ctypes.POINTER(ctypes.c_int), pu64, pu64]
    L.vcfc_query_buffer.argtypes = [vp, vp, u64, ctypes.c_char_p, u64, ctypes.c_int, u64, u64, vp, u64, pu64]
    L.vcfc_query_file.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, u64, ctypes.c_int, u64, u64, ctypes.c_int]
    L.vcfc_decode_selected_device.argtypes = [vp, u64, vp, vp, u64, u64, vp, u64, vp, vp, u64, vp, ctypes.c_int, vp]
    L.vcfc_query_match_device.argtypes = [vp, vp, u64, vp, u64, ctypes.c_int, u64, u64, vp, vp, vp]
    L.vcfc_sparse_query_file.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, u64, ctypes.c_int, u64, u64,
                                         ctypes.c_int]
    _lib = L
    return L


def strerror(st):
    return lib().vcfc_strerror(st).decode()


def raise_for(st, where=""):
    if st == OK:
        return
    msg = strerror(st) + (" (%s)" % where if where else "")
    if st in (E_LT8COLS, E_HEADER):
        raise VcfValidationError(msg)
    if st == E_8COLS:
        raise LengthError(msg)
    raise RuntimeError(msg)


class VcfCoordinateQuery(collections.namedtuple("VcfCoordinateQuery", "reference_name has_range start end")):
    """VcfCoordinateQuery (reference src/main.cpp:60-90): a reference name
    (b"" matches any) and, when has_range, an inclusive POS range."""


def parse_coordinate_string(q):
    """parse_coordinate_string (reference src/main.cpp:3993-4026), through
    the C ABI.  Raises ValueError with the reference's message where it
    prints one and returns -1."""
    qb = q.encode() if isinstance(q, str) else bytes(q)
    ref_len, has_range, start, end = ctypes.c_uint64(), ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64()
    st = lib().vcfc_parse_query(qb, len(qb), ctypes.byref(ref_len), ctypes.byref(has_range), ctypes.byref(start),
                                ctypes.byref(end))
    if st != 0:
        colon = qb.find(b":")
        dash = qb.find(b"-", colon + 1)
        msg = {1: "Query must contain a dash character: <ref>:<start>-<end>",
               2: "Failed to parse int from start position: %s" % qb[colon + 1:dash].decode(errors="replace"),
               3: "Failed to parse int from end position: %s" % qb[dash + 1:].decode(errors="replace")}.get(st)
        raise ValueError(msg or strerror(st))
    return VcfCoordinateQuery(qb[:ref_len.value], bool(has_range.value), start.value, end.value)


HOLD_CAP_DEFAULT = 32 << 30     # VCFC_HOLD_GB unset: at most 32 GiB held per rank
INGEST_PINNED_BYTES = 1 << 30   # a rank's own pinned ingest slots and staging (3 x 128 MiB + margin)


def mem_available(meminfo="/proc/meminfo"):
    """MemAvailable of this host in bytes (None when it cannot be read)."""
    try:
        with open(meminfo) as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return int(line.split()[1]) * 1024
    except OSError:
        pass
    return None


def hold_bytes(local_world=None, avail=None):
    """How much output one rank may hold in host memory before it spills
    (Context.compress_range_held's mem_bound): a share of the host's available
    memory -- 3/4 of MemAvailable split over the node's ranks, less each rank's
    pinned ingest buffers -- capped by VCFC_HOLD_GB (default 32 GiB), and at
    least 64 MiB (one hold block).  Bounding by the host, not a constant,
    keeps 8 ranks from overcommitting a node into the OOM killer while their
    peers wait in the all-gather."""
    import os
    if local_world is None:
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")) or 1)
    env = os.environ.get("VCFC_HOLD_GB")
    cap = int(float(env) * (1 << 30)) if env else HOLD_CAP_DEFAULT
    avail = mem_available() if avail is None else avail
    if avail is not None:
        cap = min(cap, (avail * 3 // 4) // max(1, local_world) - INGEST_PINNED_BYTES)
    return max(64 << 20, cap)


class Held:
    """Output of Context.compress_range_held, placed once its offset is known.
    Owns host memory (up to its bound) and a spill file: free() releases them,
    as do `with` and garbage collection."""

    def __init__(self, h):
        self._h = h

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.free()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def place(self, fd, off):
        """Write every held byte at file offset `off` of fd; returns the status."""
        return lib().vcfc_held_place(self._h, fd, off) if self._h else E_ARG

    def sizes(self):
        m, sp = ctypes.c_uint64(0), ctypes.c_uint64(0)
        lib().vcfc_held_sizes(self._h, ctypes.byref(m), ctypes.byref(sp))
        return m.value, sp.value

    def free(self):
        if self._h:
            lib().vcfc_held_free(self._h)
            self._h = None


class Context:
    """One GPU (device ordinal).  Raises if no GPU is visible."""

    def __init__(self, device=0):
        self._h = ctypes.c_void_p()
        st = lib().vcfc_ctx_create(device, ctypes.byref(self._h))
        if st != OK:
            raise RuntimeError("vcfc: cannot create a GPU context: " + strerror(st))

    def close(self):
        if self._h:
            lib().vcfc_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_ingest_chunk(self, chunk_bytes):
        """Input chunk of compress_file / compress_buffer (0 = default 128 MiB);
        the output does not depend on it."""
        raise_for(lib().vcfc_ctx_set_ingest_chunk(self._h, int(chunk_bytes)))

    def set_line_index(self, mode):
        """compress_device's line index: "hop" (default; guessed line ends,
        checked) or "scan" (every byte).  The output does not depend on it."""
        raise_for(_need("vcfc_ctx_set_line_index")(self._h, {"hop": LINE_INDEX_HOP, "scan": LINE_INDEX_SCAN}[mode]))

    def set_deferred_records(self, on):
        """Deferred records for the file / device compress calls (on by
        default since round 5): rows whose first genotype chunk is all
        escapes are sized first and written straight into the output
        (include/vcfc.h).  The output does not depend on it."""
        raise_for(_need("vcfc_ctx_set_deferred_records")(self._h, 1 if on else 0))

    def set_trace(self, flags):
        """Stage timings of the host drivers to stderr (TRACE_* flags)."""
        raise_for(_need("vcfc_ctx_set_trace")(self._h, int(flags)))

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- reference interface ------------------------------------------------
    def compress_data_line(self, line, add_newline=True):
        """bytes line (no '\\n') -> record bytes, as compress_data_line."""
        cap = lib().vcfc_encode_bound(1, len(line)) + 16
        buf = ctypes.create_string_buffer(cap)
        n = ctypes.c_uint64(0)
        st = lib().vcfc_compress_data_line(self._h, line, len(line), int(add_newline), buf, cap, ctypes.byref(n))
        raise_for(st)
        return buf.raw[:n.value]

    def compress_buffer(self, data):
        """Whole VCF (bytes) -> .vcfc bytes, as compress()."""
        cap = lib().vcfc_compress_bound(len(data))
        out = np.empty(cap, dtype=np.uint8)
        n = ctypes.c_uint64(0)
        line = ctypes.c_int64(-1)
        src = np.frombuffer(data, dtype=np.uint8)
        st = lib().vcfc_compress_buffer(self._h, src.ctypes.data, len(data), out.ctypes.data, cap,
                                        ctypes.byref(n), ctypes.byref(line))
        raise_for(st, "line %d" % line.value)
        return out[:n.value].tobytes()

    def compress_device(self, d_in, n, d_out, out_cap):
        """compress() over file bytes in device memory (pointers): d_in[0, n)
        -> d_out; returns (status, out_len, err_line) without raising."""
        k = ctypes.c_uint64(0)
        line = ctypes.c_int64(-1)
        st = lib().vcfc_compress_device(self._h, d_in, n, d_out, out_cap, ctypes.byref(k), ctypes.byref(line))
        return st, k.value, line.value

    def compress_status(self, data):
        """Like compress_buffer without raising: (status, bytes, err_line).
        On a failing line the bytes are everything the reference writes
        before it throws; err_line is its 1-based line number."""
        cap = lib().vcfc_compress_bound(len(data))
        out = np.empty(cap, dtype=np.uint8)
        n = ctypes.c_uint64(0)
        line = ctypes.c_int64(-1)
        src = np.frombuffer(data, dtype=np.uint8)
        st = lib().vcfc_compress_buffer(self._h, src.ctypes.data, len(data), out.ctypes.data, cap,
                                        ctypes.byref(n), ctypes.byref(line))
        return st, out[:n.value].tobytes(), line.value

    def compress_file(self, in_path, out_path):
        line = ctypes.c_int64(-1)
        st = lib().vcfc_compress_file(self._h, in_path.encode(), out_path.encode(), ctypes.byref(line))
        raise_for(st, "line %d" % line.value)

    def compress_range(self, in_path, off, length, out_fd, out_off=0):
        """One shard of a sharded compress: bytes [off, off + length) of
        in_path (whole lines) -> out_fd at out_off.  Returns (status,
        bytes written, 1-based failing line in the range or -1, lines in the
        range); does not raise (ranks exchange statuses first)."""
        nb, line, lines = ctypes.c_uint64(0), ctypes.c_int64(-1), ctypes.c_uint64(0)
        st = lib().vcfc_compress_range(self._h, in_path.encode(), off, length, out_fd, out_off, ctypes.byref(nb),
                                       ctypes.byref(line), ctypes.byref(lines))
        return st, nb.value, line.value, lines.value

    def compress_range_held(self, in_path, off, length, mem_bound=None, spill_dir=None):
        """compress_range with the output held (host memory up to mem_bound
        bytes -- default hold_bytes(), this rank's share of the host -- the
        rest in a spill file) until its file offset is known.
        Returns (status, bytes, failing line in the range or -1, lines in the
        range, Held); does not raise."""
        if mem_bound is None:
            mem_bound = hold_bytes()
        nb, line, lines, h = ctypes.c_uint64(0), ctypes.c_int64(-1), ctypes.c_uint64(0), ctypes.c_void_p()
        st = lib().vcfc_compress_range_held(self._h, in_path.encode(), off, length, mem_bound,
                                            spill_dir.encode() if spill_dir else None, ctypes.byref(h),
                                            ctypes.byref(nb), ctypes.byref(line), ctypes.byref(lines))
        return st, nb.value, line.value, lines.value, Held(h.value)

    def decompress_buffer(self, data, cap=None):
        """.vcfc bytes -> VCF bytes, as decompress2_fd (reference
        src/compress.cpp:1214-1257).  Returns (status, bytes): on
        VCFC_E_FORMAT the bytes are what the reference writes before it
        throws."""
        src = np.frombuffer(data, dtype=np.uint8)
        cap = cap if cap is not None else 16 * len(data) + 4096
        while True:
            out = np.empty(max(cap, 1), dtype=np.uint8)
            n = ctypes.c_uint64(0)
            st = lib().vcfc_decompress_buffer(self._h, src.ctypes.data, len(data), out.ctypes.data, cap,
                                              ctypes.byref(n))
            if st == E_NOSPACE and n.value > cap:
                cap = n.value
                continue
            return st, out[:n.value].tobytes()

    def decompress(self, data):
        """Like decompress_buffer, raising where the reference throws."""
        st, out = self.decompress_buffer(data)
        raise_for(st)
        return out

    def decompress_file(self, in_path, out_path):
        raise_for(lib().vcfc_decompress_file(self._h, in_path.encode(), out_path.encode()))

    def query_buffer(self, data, query, cap=None):
        """query_compressed_file (reference src/main.cpp:3777-3929) over .vcfc
        bytes: the matching lines (no header).  `query` is a
        VcfCoordinateQuery or a coordinate string.  Returns (status, bytes):
        on VCFC_E_FORMAT the bytes are every line the reference writes before
        it throws."""
        if not isinstance(query, VcfCoordinateQuery):
            query = parse_coordinate_string(query)
        src = np.frombuffer(data, dtype=np.uint8)
        cap = cap if cap is not None else 16 * len(data) + 4096
        while True:
            out = np.empty(max(cap, 1), dtype=np.uint8)
            n = ctypes.c_uint64(0)
            st = lib().vcfc_query_buffer(self._h, src.ctypes.data, len(data), query.reference_name,
                                         len(query.reference_name), int(query.has_range), query.start, query.end,
                                         out.ctypes.data, cap, ctypes.byref(n))
            if st == E_NOSPACE and n.value > cap:
                cap = n.value
                continue
            return st, out[:n.value].tobytes()

    def query(self, data, query):
        """Like query_buffer, raising where the reference throws."""
        st, out = self.query_buffer(data, query)
        raise_for(st)
        return out

    def query_file(self, in_path, query, out_fd=1):
        """Matching lines of a .vcfc file written to out_fd (stdout by
        default), as `main query <file> <query>`."""
        if not isinstance(query, VcfCoordinateQuery):
            query = parse_coordinate_string(query)
        raise_for(lib().vcfc_query_file(self._h, in_path.encode(), query.reference_name, len(query.reference_name),
                                        int(query.has_range), query.start, query.end, out_fd))

    def sparse_query_status(self, in_path, query):
        """query_sparse_file_fd (reference src/main.cpp:235-582) over a sparse
        file: (status, stdout bytes); E_FORMAT where the reference throws (the
        bytes are every line it writes before)."""
        import tempfile
        if not isinstance(query, VcfCoordinateQuery):
            query = parse_coordinate_string(query)
        with tempfile.TemporaryFile() as f:
            st = lib().vcfc_sparse_query_file(self._h, in_path.encode(), query.reference_name,
                                              len(query.reference_name), int(query.has_range), query.start,
                                              query.end, f.fileno())
            f.seek(0)
            return st, f.read()

    def sparse_query_file(self, in_path, query, out_fd=1):
        """Lines of a sparse file written to out_fd, as `main sparse-query`."""
        if not isinstance(query, VcfCoordinateQuery):
            query = parse_coordinate_string(query)
        raise_for(lib().vcfc_sparse_query_file(self._h, in_path.encode(), query.reference_name,
                                               len(query.reference_name), int(query.has_range), query.start,
                                               query.end, out_fd))

    def sparsify_file(self, in_path, out_path):
        """sparsify_file (reference src/sparse.cpp:290-580)."""
        raise_for(lib().vcfc_sparsify_file(self._h, in_path.encode(), out_path.encode()))

    def sparsify_status(self, in_path, out_path):
        """sparsify_file without raising: the C status (VCFC_E_FORMAT where the
        reference throws, after writing the records before)."""
        return lib().vcfc_sparsify_file(self._h, in_path.encode(), out_path.encode())

    def sparsify_shard(self, in_path, out_path, rank, world):
        """This rank's slice of a sharded sparsify (vcfc_sparsify_shard):
        out_path None plans only.  Returns (status, [lo, hi, first_err or
        None, anomaly])."""
        info = (ctypes.c_uint64 * 4)()
        st = lib().vcfc_sparsify_shard(self._h, in_path.encode(), out_path.encode() if out_path else None,
                                       rank, world, info)
        return st, [info[0], info[1], None if info[2] == NO_ERROR else info[2], info[3]]

    def encode_rows(self, buf, line_off, line_len):
        """Host batch: returns (status, records bytes, rec_off, err_row)."""
        n = len(line_off)
        lo = np.ascontiguousarray(line_off, dtype=np.uint64)
        ll = np.ascontiguousarray(line_len, dtype=np.uint32)
        src = np.frombuffer(buf, dtype=np.uint8)
        cap = lib().vcfc_encode_bound(n, int(ll.sum(dtype=np.uint64))) + 16
        out = np.empty(cap, dtype=np.uint8)
        rec = np.zeros(n + 1, dtype=np.uint64)
        er = ctypes.c_int64(-1)
        st = lib().vcfc_encode_rows(self._h, src.ctypes.data, len(buf), lo.ctypes.data, ll.ctypes.data, n,
                                    out.ctypes.data, cap, rec.ctypes.data, ctypes.byref(er))
        upto = n if st == OK else max(er.value, 0)
        return st, out[:int(rec[upto])].tobytes(), rec, er.value


# -- device-pointer API (used with torch tensors in bench.py / GPU tests) ----
def workspace_size(n_rows, total_line_bytes):
    return int(lib().vcfc_encode_workspace_size(n_rows, total_line_bytes))


def encode_bound(n_rows, total_line_bytes):
    return int(lib().vcfc_encode_bound(n_rows, total_line_bytes))


def encode_rows_device(d_buf, d_line_off, d_line_len, n, total_line_bytes, d_out, out_cap, d_rec_off,
                       d_ws, ws_bytes, d_err, stream=0):
    st = lib().vcfc_encode_rows_device(d_buf, d_line_off, d_line_len, n, total_line_bytes, d_out, out_cap,
                                       d_rec_off, d_ws, ws_bytes, d_err, stream)
    raise_for(st)


def _need(name):
    """The export `name` of the loaded library (an older build loaded through
    VCFC_LIB may lack it: a clear error instead of an AttributeError)."""
    L = lib()
    if not hasattr(L, name):
        raise RuntimeError("%s: %s is not exported by this build of libvcfc.so" % (LIB_PATH, name))
    return getattr(L, name)


def encode_deferred_rows(d_ws, n, total_line_bytes, stream=0):
    """Rows the last encode_rows_device on workspace d_ws deferred (waits for stream)."""
    v = ctypes.c_uint64(0)
    raise_for(_need("vcfc_encode_deferred_rows")(d_ws, n, total_line_bytes, stream, ctypes.byref(v)))
    return int(v.value)


class StageTimer:
    """Per-stage HIP-event timing of encode_rows_device (see vcfc_timer_read)."""
    STAGES = ("slot_scan", "k_encode", "size_scan", "k_compact")

    def __init__(self):
        self._h = ctypes.c_void_p()
        raise_for(lib().vcfc_timer_create(ctypes.byref(self._h)))

    def encode(self, d_buf, d_line_off, d_line_len, n, total_line_bytes, d_out, out_cap, d_rec_off,
               d_ws, ws_bytes, d_err, stream=0):
        raise_for(lib().vcfc_encode_rows_device_timed(d_buf, d_line_off, d_line_len, n, total_line_bytes, d_out,
                                                      out_cap, d_rec_off, d_ws, ws_bytes, d_err, stream, self._h))

    def read(self):
        ms = (ctypes.c_double * 4)()
        calls = ctypes.c_uint64(0)
        raise_for(lib().vcfc_timer_read(self._h, ms, ctypes.byref(calls)))
        return dict(zip(self.STAGES, list(ms))), calls.value

    def __del__(self):
        try:
            lib().vcfc_timer_destroy(self._h)
        except Exception:
            pass


def decode_workspace_size(n_records):
    return int(lib().vcfc_decode_workspace_size(n_records))


def decode_records_device(d_in, in_bytes, d_rec_start, n, samples, d_out, out_cap, d_line_off, d_ws, ws_bytes,
                          d_err, stream=0, exact=False):
    raise_for(lib().vcfc_decode_records_device(d_in, in_bytes, d_rec_start, n, samples, d_out, out_cap, d_line_off,
                                               d_ws, ws_bytes, d_err, int(exact), stream))


def decode_selected_device(d_in, in_bytes, d_rec_start, d_select, n, samples, d_out, out_cap, d_line_off, d_ws,
                           ws_bytes, d_err, stream=0, exact=False):
    raise_for(lib().vcfc_decode_selected_device(d_in, in_bytes, d_rec_start, d_select, n, samples, d_out, out_cap,
                                                d_line_off, d_ws, ws_bytes, d_err, int(exact), stream))


def query_match_device(d_in, d_rec_start, n, d_ref, ref_len, has_range, start, end, d_flag, d_err, stream=0):
    """Device match step of the range query (see include/vcfc.h)."""
    return lib().vcfc_query_match_device(d_in, d_rec_start, n, d_ref, ref_len, int(has_range), start, end, d_flag,
                                         d_err, stream)


def synth_rows_device(d_buf, d_line_off, n, d_prefix, d_prefix_off, d_row_af, samples, law, seed, stream=0,
                      row_base=0):
    st = lib().vcfc_synth_rows_device_at(d_buf, d_line_off, n, d_prefix, d_prefix_off, d_row_af, samples,
                                         law, seed, row_base, stream)
    raise_for(st)


def record_hash_device(d_recs, d_rec_off, n, d_hash, stream=0):
    """Per-record 64-bit digests on the GPU (include/vcfc.h vcfc_record_hash_device)."""
    raise_for(lib().vcfc_record_hash_device(d_recs, d_rec_off, n, d_hash, stream))
