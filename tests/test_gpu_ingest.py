"""GPU parity of the pipelined file compress (reference
compress(), src/compress.cpp:205-257, which streams the file with getline).

The multi-chunk path runs on real HIP streams here: the input chunk is forced
down to 4 KiB / 1 MiB / 16 MiB (vcfc_ctx_set_ingest_chunk), so reader
threads, three pinned input slots, two device slots, the uploader stream and
its events, partial lines carried across chunks and chunks grown around long
lines all run on the GPU.  Every case also runs through vcfc_compress_device
(the same file bytes resident in device memory, chunked the same way).  Outputs are checked byte for byte against the
reference's own compress outputs (tests/golden) and against the oracle; the
300 MiB case against the device encoder's records of the same rows."""
import os
import random
import tempfile

import numpy as np
import pytest

import decode_cases as D
import golden_io as G

pytestmark = pytest.mark.gpu
REPO = G.REPO
CHUNKS = [4096, 1 << 20, 16 << 20]


@pytest.fixture(scope="module")
def torch():
    import torch as T   # before libvcfc: one HIP runtime in the process
    assert T.cuda.is_available(), "GPU tests need a GPU"
    return T


@pytest.fixture(scope="module")
def vcfc(torch):
    import sys
    sys.path.insert(0, os.path.join(REPO, "vcf-compression_amd"))
    import vcfc as V
    return V


@pytest.fixture(scope="module")
def ctx(vcfc):
    c = vcfc.Context(0)
    yield c
    c.close()


def device_path(ctx, data):
    """(status, bytes, err_line) from vcfc_compress_device: the file bytes
    already in device memory (an unterminated last line gets its '\n', as
    getline returns it), line index + encode on the GPU, output in HBM."""
    import torch as T
    import vcfc as V
    if data and not data.endswith(b"\n"):
        data = data + b"\n"
    d_in = T.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).to("cuda:0") if data else \
        T.empty(16, dtype=T.uint8, device="cuda:0")
    cap = int(V.lib().vcfc_compress_bound(len(data)))
    d_out = T.empty(cap, dtype=T.uint8, device="cuda:0")
    T.cuda.synchronize()   # the call runs on the context's own stream
    st, k, el = ctx.compress_device(d_in.data_ptr(), len(data), d_out.data_ptr(), cap)
    return st, d_out[:k].cpu().numpy().tobytes(), el


def both_paths(ctx, data, chunk):
    """(status, bytes, err_line) from compress_buffer (memory source), from
    compress_file (fd source, pread by reader threads) and from
    compress_device (device-resident bytes); they must agree."""
    ctx.set_ingest_chunk(chunk)
    try:
        st, out, el = ctx.compress_status(data)
        with tempfile.TemporaryDirectory(dir="/tmp") as d:
            ip, op = os.path.join(d, "in.vcf"), os.path.join(d, "out.vcfc")
            with open(ip, "wb") as f:
                f.write(data)
            import ctypes
            line = ctypes.c_int64(-1)
            from vcfc import lib
            st2 = lib().vcfc_compress_file(ctx._h, ip.encode(), op.encode(), ctypes.byref(line))
            out2 = open(op, "rb").read()
        assert (st2, out2, line.value) == (st, out, el), (chunk, st, st2, len(out), len(out2))
        st3, out3, el3 = device_path(ctx, data)
        assert (st3, out3, el3) == (st, out, el), (chunk, st, st3, len(out), len(out3))
        return st, out, el
    finally:
        ctx.set_ingest_chunk(0)


@pytest.mark.parametrize("chunk", CHUNKS)
def test_config1_multi_chunk(ctx, chunk):
    st, out, _ = both_paths(ctx, G.gz("random_100x10000.vcf.gz"), chunk)
    assert st == 0 and out == G.gz("random_100x10000.vcfc.gz")


@pytest.mark.parametrize("chunk", CHUNKS)
def test_fuzz_corpus_multi_chunk(ctx, chunk):
    st, out, _ = both_paths(ctx, G.gz("fuzz_encode.vcf.gz"), chunk)
    assert st == 0 and out == G.gz("fuzz_encode.vcfc.gz")


@pytest.mark.parametrize("chunk", CHUNKS)
def test_edge_file_multi_chunk(ctx, chunk):
    ec = G.edge_cases()
    st, out, _ = both_paths(ctx, bytes.fromhex(ec["file"]["input"]), chunk)
    assert st == 0 and out.hex() == ec["file"]["output"]
    data = bytes.fromhex(ec["bad_header_file"]["input"])
    assert both_paths(ctx, data, chunk) == G.oracle_compress(data)


def test_errors_straddling_chunks(ctx):
    """A failing line (< 8 columns, exactly 8, a '#' header line with < 8
    terms) inserted at every 23rd line of a 400 KB prefix of config-1 and read
    in 4 KiB chunks (~10 lines each, so many insertions straddle a chunk
    boundary): the status, the 1-based line number and every byte written
    before it match the oracle."""
    vcf = G.gz("random_100x10000.vcf.gz")[: 400_000]
    vcf = vcf[: vcf.rindex(b"\n") + 1]
    starts = [0] + [i + 1 for i, c in enumerate(vcf) if c == 10][:-1]
    bad = [b"1\t2\t3", b"1\t2\t3\t4\t5\t6\t7\t8", b"#CHROM\tPOS"]
    for k, b in enumerate(bad):
        for at in starts[3 + k::23]:
            data = vcf[:at] + b + b"\n" + vcf[at:]
            want = G.oracle_compress(data)
            assert want[0] != 0
            assert both_paths(ctx, data, 4096) == want, (b, at)


def test_long_lines_grow_the_chunk(ctx):
    """Lines longer than the chunk (up to 9x) between short ones: the chunk
    grows around them; output equals the oracle's."""
    rnd = random.Random(3)
    lines = D.header(40).rstrip(b"\n").split(b"\n") + D.rows(rnd, 30, 40, escapes=0.03)
    for k, n in enumerate([3000, 9000, 1200]):
        toks = [rnd.choice([b"0|0", b"0|1", b"1|1", b"0|2"]) for _ in range(n)]
        lines.insert(5 + 10 * k, b"\t".join([b"1", b"%d" % k, b"a", b"b", b"c", b"d", b"e", b"f", b"GT"] + toks))
    data = b"\n".join(lines)   # unterminated last line
    st_o, want, _ = G.oracle_compress(data)
    assert st_o == 0
    assert both_paths(ctx, data, 4096) == (0, want, -1)


def test_300mib_chr22_file_multi_chunk(torch, vcfc, ctx):
    """>= 300 MiB of chr22-shaped rows (2504 samples) with '#' and empty lines
    interleaved, through 16 MiB and 7 MiB + 1 B chunks (~20-45 chunks: slot
    rotation, copy/compute overlap, carries): the output equals the header +
    the device encoder's records of the same rows (sampled rows also checked
    against the oracle)."""
    import workload
    from test_gpu_encode import _device_encode
    n = 32_000
    rows = workload.DeviceRows(torch, vcfc, n, 2504, 1, seed=21, device="cuda:0")
    out, rec, err = _device_encode(torch, vcfc, rows)
    assert err == vcfc.NO_ERROR
    recs = out[:int(rec[n])].cpu().numpy().tobytes()
    body = rows.buf[:rows.total_bytes].cpu().numpy().tobytes()
    lo = rows.line_off.cpu().numpy()
    hdr = D.header(2504)
    # pass-through lines at a few row boundaries (and an empty line)
    parts, want, prev = [hdr], [hdr], 0
    for i in list(range(997, n, 2741)) + [n]:
        parts.append(body[int(lo[prev]):int(lo[i]) if i < n else len(body)])
        want.append(recs[int(rec[prev]):int(rec[i])])
        if i < n:
            note = b"##note row %d\n" % i
            parts.append(note + b"\n")
            want.append(note)
        prev = i
    data = b"".join(parts)
    nbytes = len(data)
    assert nbytes >= 300 << 20, nbytes
    want = b"".join(want)
    for chunk in (16 << 20, (7 << 20) + 1):
        st, got, el = both_paths(ctx, data, chunk)
        assert st == 0 and el == -1
        assert len(got) == len(want) and got == want, chunk
    pick = np.random.default_rng(1).integers(0, n, 40)
    for i, ln in zip(pick, rows.host_lines(pick)):
        assert recs[int(rec[i]):int(rec[i + 1])] == G.oracle_encode_line(ln)[1], i


@pytest.mark.parametrize("kind", ["tab", "escape", "var", "lines"])
def test_hop_index_wrong_guess_on_gpu(ctx, kind):
    """The hop line index's traps (tests/hop_cases.py: a row shorter than the
    header's sample count whose guessed end is a later row's '\\n') on the
    GPU: the encoder's '\\n' check sends the chunk back to the full scan, and
    the output is the oracle's -- whole file and 4 KiB chunks (every path of
    both_paths)."""
    from hop_cases import hop_trap_file
    data = hop_trap_file(kind, random.Random(kind))
    st_o, want, _ = G.oracle_compress(data)
    assert st_o == 0
    assert both_paths(ctx, data, 1 << 20) == (0, want, -1)
    assert both_paths(ctx, data, 4096) == (0, want, -1)


def test_hop_index_chr22_like_on_gpu(ctx):
    """chr22-shaped rows whose prefix lengths jump by up to 300 bytes (guess
    windows that miss and the VERIFY round), '##' and empty lines between
    them: device path equals the oracle."""
    from hop_cases import chr22_like
    for S, jitter in ((300, 40), (700, 300), (64, 5)):
        data = chr22_like(random.Random(S), 150, S, jitter)
        st_o, want, _ = G.oracle_compress(data)
        assert st_o == 0 and both_paths(ctx, data, 1 << 20) == (0, want, -1), S


def test_hop_index_wrong_guess_in_dense_segment_on_gpu(ctx):
    """A wrong guess in a 16 KiB segment of more than 128 line ends whose last
    line is a '#' line (hop_cases.hop_trap_dense_segment): k_nl_place's
    rescan finds the hop's count short and the chunk is indexed again; the
    '#' line is not written with a data row inside it."""
    from hop_cases import hop_trap_dense_segment
    data = hop_trap_dense_segment(random.Random(5))
    st_o, want, _ = G.oracle_compress(data)
    assert st_o == 0
    assert both_paths(ctx, data, 1 << 20) == (0, want, -1)


@pytest.mark.parametrize("chunk", [1 << 16, 16 << 20])
def test_law2_like_deferred_records_on_gpu(ctx, chunk):
    """Deferred records (vcfc_ctx_set_deferred_records) through all three
    ingest paths -- buffer, file, device-resident bytes -- on law-2-shaped
    files (GT:DP:GQ rows of fixed and of random widths beside haploid and
    missing rows): the oracle's output, and the same bytes as without."""
    from hop_cases import law2_like
    for S, dp in ((700, 2), (2504, 0)):
        vcf = law2_like(random.Random(S + dp), 40, S, dp_width=dp)
        st_o, want, _ = G.oracle_compress(vcf)
        assert st_o == 0
        ctx.set_deferred_records(True)
        try:
            st, out, el = both_paths(ctx, vcf, chunk)
        finally:
            ctx.set_deferred_records(False)
        assert (st, el) == (0, -1) and out == want, (S, dp, chunk)
