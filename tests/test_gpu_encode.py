"""GPU parity: the HIP path (through the C ABI) against the reference's golden
vectors and the oracle.  Needs a gfx950 GPU (-m gpu)."""
import hashlib
import io
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu
REPO = G.REPO
sys.path.insert(0, os.path.join(REPO, "vcf-compression_amd"))


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def torch():
    import torch as T   # import before libvcfc: one HIP runtime in the process
    assert T.cuda.is_available(), "GPU tests need a GPU"
    return T


@pytest.fixture(scope="module")
def vcfc(torch):
    import vcfc as V
    return V


@pytest.fixture(scope="module")
def ctx(vcfc):
    c = vcfc.Context(0)
    yield c
    c.close()


def test_edge_cases_known_answers(ctx, vcfc):
    for case in G.edge_cases()["cases"]:
        line = bytes.fromhex(case["line"])
        if "record" in case:
            assert ctx.compress_data_line(line).hex() == case["record"], case["name"]
        elif case["error"] == "length_error":
            with pytest.raises(vcfc.LengthError):
                ctx.compress_data_line(line)
        else:
            with pytest.raises(vcfc.VcfValidationError):
                ctx.compress_data_line(line)


def test_compress_data_line_without_newline(ctx):
    line = bytes.fromhex(G.edge_cases()["cases"][0]["line"])
    st, want = G.oracle_encode_line(line, add_newline=False)
    assert st == 0 and ctx.compress_data_line(line, add_newline=False) == want


def test_edge_file_and_bad_header(ctx, vcfc):
    ec = G.edge_cases()
    assert ctx.compress_buffer(bytes.fromhex(ec["file"]["input"])).hex() == ec["file"]["output"]
    with pytest.raises(vcfc.VcfValidationError):
        ctx.compress_buffer(bytes.fromhex(ec["bad_header_file"]["input"]))


def test_config1_random_100x10000(ctx):
    m = G.manifest()["random_100x10000"]
    out = ctx.compress_buffer(G.gz("random_100x10000.vcf.gz"))
    assert sha(out) == m["vcfc_sha256"]


def test_fuzz_corpus(ctx):
    assert ctx.compress_buffer(G.gz("fuzz_encode.vcf.gz")) == G.gz("fuzz_encode.vcfc.gz")


def test_random_2504x4000_sha256(ctx):
    import random_vcf
    m = G.manifest()["random_2504x4000"]
    buf = io.BytesIO()
    random_vcf.generate(2504, 4000, buf)
    vcf = buf.getvalue()
    assert sha(vcf) == m["vcf_sha256"]
    assert sha(ctx.compress_buffer(vcf)) == m["vcfc_sha256"]


def test_cli_compress_matches_reference_bytes():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "t.vcf")
        with open(src, "wb") as f:
            f.write(G.gz("random_100x10000.vcf.gz"))
        r = subprocess.run([os.path.join(REPO, "build", "main"), "compress", src, src + ".vcfc"],
                           capture_output=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert sha(open(src + ".vcfc", "rb").read()) == G.manifest()["random_100x10000"]["vcfc_sha256"]


def _device_encode(torch, vcfc, rows):
    n = rows.n
    ws_bytes = vcfc.workspace_size(n, rows.line_bytes)
    cap = vcfc.encode_bound(n, rows.line_bytes)
    dev = rows.buf.device
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    rec = torch.empty(n + 1, dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    vcfc.encode_rows_device(rows.buf.data_ptr(), rows.line_off.data_ptr(), rows.line_len.data_ptr(), n,
                            rows.line_bytes, out.data_ptr(), cap, rec.data_ptr(), ws.data_ptr(), ws_bytes,
                            err.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return out, rec.cpu().numpy().astype(np.uint64), int(err.cpu().numpy().view(np.uint64)[0])


@pytest.mark.parametrize("law,samples,n", [(0, 2504, 3000), (1, 2504, 3000), (0, 100, 20000), (1, 5003, 700),
                                           (2, 2504, 3000), (2, 100, 20000), (2, 7, 5000), (3, 2504, 3000),
                                           (3, 5, 4000), (1, 100_000, 48), (0, 100_000, 24)])   # last two: configs[3] rows
def test_synthetic_rows_all_vs_oracle(torch, vcfc, law, samples, n):
    import workload
    rows = workload.DeviceRows(torch, vcfc, n, samples, law, seed=7 + law, device="cuda:0")
    out, rec, err = _device_encode(torch, vcfc, rows)
    assert err == vcfc.NO_ERROR
    host = out[:int(rec[n])].cpu().numpy().tobytes()
    lines = rows.host_lines(range(n))
    for i, ln in enumerate(lines):
        st, want = G.oracle_encode_line(ln)
        assert st == 0
        assert host[int(rec[i]):int(rec[i + 1])] == want, i


def test_config2_full_size_sampled(torch, vcfc):
    """2504 x 1M chr22-shaped rows: sampled rows byte-exact vs the oracle, and
    the record offsets consistent with every record's own LEN header."""
    import workload
    n = 1_000_000
    rows = workload.DeviceRows(torch, vcfc, n, 2504, 1, seed=11, device="cuda:0")
    out, rec, err = _device_encode(torch, vcfc, rows)
    assert err == vcfc.NO_ERROR
    sizes = np.diff(rec)
    # LEN header of every record == size - 4 (checked on device)
    rt = torch.from_numpy(rec[:-1].astype(np.int64)).cuda()
    hdr = torch.stack([out[rt + k].to(torch.int64) for k in range(4)], 1)
    L = ((hdr[:, 0] & 0x3F) << 24) | (hdr[:, 1] << 16) | (hdr[:, 2] << 8) | hdr[:, 3]
    assert bool(((hdr[:, 0] & 0xC0) == 0xC0).all())
    assert bool((L.cpu().numpy() == sizes.astype(np.int64) - 4).all())
    last = out[rt + torch.from_numpy(sizes.astype(np.int64)).cuda() - 1]
    assert bool((last == 10).all())
    rng = np.random.default_rng(5)
    pick = np.unique(np.concatenate([rng.integers(0, n, 400), [0, n - 1]]))
    lines = rows.host_lines(pick)
    for i, ln in zip(pick, lines):
        st, want = G.oracle_encode_line(ln)
        got = out[int(rec[i]):int(rec[i + 1])].cpu().numpy().tobytes()
        assert got == want, i


@pytest.mark.parametrize("name,key", [("random_100x10000.vcfc.gz", "sparse_100x10000"),
                                      ("sparse_edge.vcfc.gz", "sparse_edge")])
def test_sparsify_matches_reference(ctx, name, key):
    import sparse_digest
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.vcfc"), os.path.join(d, "out.sparse")
        with open(src, "wb") as f:
            f.write(G.gz(name))
        ctx.sparsify_file(src, dst)
        assert sparse_digest.digest(dst) == G.manifest()[key]
        r = subprocess.run([os.path.join(REPO, "build", "main"), "sparsify", src, dst + "2"],
                           capture_output=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert sparse_digest.digest(dst + "2") == G.manifest()[key]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_logical_shards_stitch_on_one_gpu(vcfc, world):
    """the multi-GPU stitch with 1/2/4/8 logical shards on one
    device (one thread and one context per shard, a fake all-gather): the
    output is byte-identical to the reference's for every shard count."""
    import threading
    import dist_compress as D
    data = G.gz("random_100x10000.vcf.gz")
    want = G.gz("random_100x10000.vcfc.gz")
    with tempfile.TemporaryDirectory() as d:
        ip, op = os.path.join(d, "in.vcf"), os.path.join(d, "out.vcfc")
        with open(ip, "wb") as f:
            f.write(data)
        open(op, "wb").close()
        slots, bar, res = [None] * world, threading.Barrier(world), [None] * world

        def worker(rank):
            with vcfc.Context(0) as ctx:
                def allgather(vals):
                    slots[rank] = vals
                    bar.wait()
                    out = list(slots)
                    bar.wait()   # (the next all-gather reuses the slots)
                    return out

                def hold(p, off, length):
                    return ctx.compress_range_held(p, off, length, spill_dir=d)
                res[rank] = D.compress_shard(ip, op, rank, world, ctx.compress_range, hold, allgather)

        ts = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        assert all(r is not None and r[0] == 0 for r in res), res
        assert open(op, "rb").read() == want


@pytest.mark.parametrize("seed", [51, 52, 53, 54])
def test_variable_token_rows(ctx, seed):
    """k_encode_var on the GPU: rows of odd-length tokens (haploid beside
    diploid, '.', GT:DP:GQ, 41-byte tokens, all-1-byte rows, long runs broken
    by 1-byte escapes) plus rows it must hand on (even-length tokens, empty
    fields, a trailing TAB, CR, a failure in the third chunk), through
    compress_buffer: byte-exact against the oracle."""
    import random
    import test_kernel_emu as T
    rnd = random.Random(seed)
    lines = T._var_rows(rnd, 120, ["hap", "dot", "long", "ones", "runs", "gdg"])
    lines += [T.PFX_V + b"0\t1|1\t10\t0|0", T.PFX_V + b"0\t\t1|1\t0", T.PFX_V + b"1\t0|0\t",
              T.PFX_V + b"\t".join([b"0"] * 2000 + [b"10", b"11", b"1"])]
    rnd.shuffle(lines)
    hdr = b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS0\n"
    data = hdr + b"\n".join(lines) + b"\n"
    st, want, _ = G.oracle_compress(data)
    assert st == 0
    assert ctx.compress_buffer(data) == want


@pytest.mark.parametrize("odd", ["none", "ntok", "mixed_later", "general_later", "long_then_plain"])
def test_predicted_deferred_records(ctx, odd):
    """GT:DP:GQ rows of one sample count: after two rows agree on their token
    count, k_encode_var sizes the later deferred rows without reading them
    (a long first token: all escapes predicted; 1-byte tokens: from their
    first chunk) and k_encode_defer's first pass checks each.  With one odd
    row among them -- a sample more, plain tokens after a first chunk of
    1-byte escapes, two even-length tokens after the first chunk (the
    general path), plain tokens right after a long first token -- the
    check fails and the gated size scan,
    compaction and deferred pass lay the batch out again: byte-exact
    against the oracle through compress_buffer either way."""
    import random
    import test_kernel_emu as T
    rnd = random.Random(hash(odd) & 0xFFFF)
    lines = [T._gdg(rnd, 700) for _ in range(300)]
    for i in range(17, 300, 61):
        if odd == "ntok":
            lines[i] = T._gdg(rnd, 701)
        elif odd == "mixed_later":
            lines[i] = T.PFX_V + b"\t".join([rnd.choice([b"0", b"1", b"."]) for _ in range(1100)] +
                                            [rnd.choice([b"0|0", b"0|1"]) for _ in range(400)])
        elif odd == "general_later":
            lines[i] = T.PFX_V + b"\t".join([b"0|1:33:99"] * 300 + [b"0|1:3:99"] * 2 + [b"0|1:33:99"] * 398)
        elif odd == "long_then_plain":
            lines[i] = T.PFX_V + b"\t".join([b"0|1:33:99"] + [rnd.choice([b"0|0", b"0|1"]) for _ in range(699)])
    hdr = (b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" +
           b"\t".join(b"S%d" % j for j in range(700)) + b"\n")
    data = hdr + b"\n".join(lines) + b"\n"
    st, want, _ = G.oracle_compress(data)
    assert st == 0
    assert ctx.compress_buffer(data) == want


def test_unphased_rows_handed_on(ctx):
    """Unphased rows ("0/1", "./.": every token of the first 2 KiB an escape)
    go from k_encode_fast to k_encode_var, which predicts their records;
    with a row that turns plain after its first chunk, one with a sample
    more, single-chunk rows and rows starting with a plain token among them:
    byte-exact against the oracle through compress_buffer."""
    import random
    import test_kernel_emu as T
    rnd = random.Random(5150)
    unph = [b"0/0", b"0/1", b"1/1", b"./."]
    S = 900
    lines = [T.PFX_V + b"\t".join(rnd.choice(unph) for _ in range(S)) for _ in range(400)]
    for i in range(13, 400, 47):
        k = rnd.randrange(4)
        if k == 0:
            lines[i] = T.PFX_V + b"\t".join([rnd.choice(unph) for _ in range(600)] +
                                            [rnd.choice([b"0|0", b"0|1"]) for _ in range(S - 600)])
        elif k == 1:
            lines[i] = T.PFX_V + b"\t".join(rnd.choice(unph) for _ in range(S + 1))
        elif k == 2:
            lines[i] = T.PFX_V + b"\t".join(rnd.choice(unph) for _ in range(200))
        else:
            lines[i] = T.PFX_V + b"\t".join([b"0|1"] + [rnd.choice(unph) for _ in range(S - 1)])
    hdr = (b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" +
           b"\t".join(b"S%d" % j for j in range(S)) + b"\n")
    data = hdr + b"\n".join(lines) + b"\n"
    st, want, _ = G.oracle_compress(data)
    assert st == 0
    assert ctx.compress_buffer(data) == want


@pytest.mark.parametrize("law", [0, 2])
def test_encode_captured_in_hip_graph(torch, vcfc, law):
    """vcfc_encode_rows_device enqueues its whole pipeline (the reset kernel,
    the two look-back scans, k_encode_fast, k_encode_var, k_compact_out, the
    deferred passes and the gated relayout) with no host synchronisation, so
    it can be captured in a HIP graph: the replayed graph writes the same
    records, offsets and status as an eager call, replay after replay (the
    workspace state is re-zeroed by the captured reset kernel).  Law 2 takes
    the deferred and predicted records (GT:DP:GQ rows)."""
    import workload
    rows = workload.DeviceRows(torch, vcfc, 2000, 2504, law, seed=41, device="cuda:0")
    n = rows.n
    want_out, want_rec, want_err = _device_encode(torch, vcfc, rows)
    ws_bytes = vcfc.workspace_size(n, rows.line_bytes)
    cap = vcfc.encode_bound(n, rows.line_bytes)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device="cuda:0")
    out = torch.zeros(cap, dtype=torch.uint8, device="cuda:0")
    rec = torch.zeros(n + 1, dtype=torch.int64, device="cuda:0")
    err = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        vcfc.encode_rows_device(rows.buf.data_ptr(), rows.line_off.data_ptr(), rows.line_len.data_ptr(), n,
                                rows.line_bytes, out.data_ptr(), cap, rec.data_ptr(), ws.data_ptr(), ws_bytes,
                                err.data_ptr(), torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert int(err.cpu().numpy().view(np.uint64)[0]) == want_err == vcfc.NO_ERROR
        r = rec.cpu().numpy().astype(np.uint64)
        assert np.array_equal(r, want_rec)
        k = int(r[n])
        assert torch.equal(out[:k], want_out[:k])


def test_mispredicted_batch_replayed_in_hip_graph(torch, vcfc):
    """A batch whose predicted deferred records are wrong (one GT:DP:GQ row
    with a sample more among rows that agree), captured in a HIP graph: every
    replay resets the misprediction word, finds the wrong size again and
    lays the batch out again through the gated launches -- records equal to
    the oracle's on each replay."""
    import random
    import test_kernel_emu as T
    rnd = random.Random(77)
    lines = [T._gdg(rnd, 700) for _ in range(200)]
    lines[150] = T._gdg(rnd, 701)
    buf = b"".join(ln + b"\n" for ln in lines)
    off = np.cumsum([0] + [len(ln) + 1 for ln in lines[:-1]]).astype(np.int64)
    ln_ = np.array([len(ln) for ln in lines], dtype=np.int32)
    dev = "cuda:0"
    d_buf = torch.from_numpy(np.frombuffer(buf + b"\0" * 64, dtype=np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.from_numpy(ln_).to(dev)
    n, tot = len(lines), int(ln_.sum())
    ws_bytes = vcfc.workspace_size(n, tot)
    cap = vcfc.encode_bound(n, tot)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    out = torch.zeros(cap, dtype=torch.uint8, device=dev)
    rec = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    err = torch.zeros(1, dtype=torch.int64, device=dev)
    want = [G.oracle_encode_line(x)[1] for x in lines]
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        vcfc.encode_rows_device(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, tot, out.data_ptr(), cap,
                                rec.data_ptr(), ws.data_ptr(), ws_bytes, err.data_ptr(),
                                torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert int(err.cpu().numpy().view(np.uint64)[0]) == vcfc.NO_ERROR
        r = rec.cpu().numpy()
        blob = out[:int(r[n])].cpu().numpy().tobytes()
        assert blob == b"".join(want)


@pytest.mark.parametrize("law,kind", [(2, "1"), (1, None), (0, None), (2, None), (2, "3")])
def test_deferred_records_chosen_per_row(torch, vcfc, monkeypatch, law, kind):
    """Deferred records are on by default (round 5) and the kernel chooses them
    per row from the row's bytes: every GT:DP:GQ row (law-2 kind 1: its first
    genotype chunk all escapes, more than one chunk) is deferred, and every
    unphased row (kind 3: a first chunk of 3-byte escapes only, which
    k_encode_fast hands on); no row of the chr22 / random_vcf laws is, and in
    the law-2 mix exactly the GT:DP:GQ and unphased rows are.  Every record
    equals the oracle's."""
    import workload
    if kind is None:
        monkeypatch.delenv("VCFC_LAW2_KIND", raising=False)
    else:
        monkeypatch.setenv("VCFC_LAW2_KIND", kind)
    n, S = 3000, 2504
    rows = workload.DeviceRows(torch, vcfc, n, S, law, seed=91 + law, device="cuda:0")
    ws_bytes = vcfc.workspace_size(n, rows.line_bytes)
    cap = vcfc.encode_bound(n, rows.line_bytes)
    dev = rows.buf.device
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    rec = torch.empty(n + 1, dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    vcfc.encode_rows_device(rows.buf.data_ptr(), rows.line_off.data_ptr(), rows.line_len.data_ptr(), n,
                            rows.line_bytes, out.data_ptr(), cap, rec.data_ptr(), ws.data_ptr(), ws_bytes,
                            err.data_ptr(), torch.cuda.current_stream().cuda_stream)
    deferred = vcfc.encode_deferred_rows(ws.data_ptr(), n, rows.line_bytes, torch.cuda.current_stream().cuda_stream)
    assert int(err.cpu().numpy().view(np.uint64)[0]) == vcfc.NO_ERROR
    lines = rows.host_lines(range(n))
    r = rec.cpu().numpy()
    blob = out[:int(r[n])].cpu().numpy().tobytes()
    for i, ln in enumerate(lines):
        st, want = G.oracle_encode_line(ln)
        assert st == 0 and blob[int(r[i]):int(r[i + 1])] == want, i
    gdg = sum(b"GT:DP:GQ" in ln for ln in lines)
    unph = sum(b"KIND=3" in ln for ln in lines)   # (law 2's INFO names the row kind)
    assert deferred == gdg + unph, (deferred, gdg, unph)
    if kind in ("1", "3"):
        assert gdg + unph == n
    elif law != 2:
        assert gdg + unph == 0
    else:
        assert 0 < gdg < n and 0 < unph < n


def test_line_longer_than_the_length_header_is_refused(torch, vcfc):
    """a data line over VCFC_MAX_LINE (2^29 - 64 bytes) could give
    a record past the 30-bit LEN header (reference src/utils.hpp:140-160) and
    past the rec_size flag bits: the encode reports VCFC_E_TOOLONG at that
    row (the rows before it are valid output) instead of a wrong record."""
    import workload
    small = workload.DeviceRows(torch, vcfc, 3, 50, 1, seed=3, device="cuda:0")
    lines = small.host_lines(range(3))
    big = lines[0] + b"\t0|0" * ((vcfc.MAX_LINE - len(lines[0])) // 4 + 1)
    assert len(big) > vcfc.MAX_LINE
    rows = [lines[0], lines[1], big, lines[2]]
    buf = bytearray()
    offs, lens = [], []
    for ln in rows:
        offs.append(len(buf))
        lens.append(len(ln))
        buf += ln + b"\n"
    dev = torch.device("cuda:0")
    d_buf = torch.from_numpy(np.frombuffer(bytes(buf), dtype=np.uint8).copy()).to(dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    d_len = torch.tensor(lens, dtype=torch.int32, device=dev)
    n, total = 4, sum(lens)
    ws_bytes = vcfc.workspace_size(n, total)
    cap = vcfc.encode_bound(n, total)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    rec = torch.empty(n + 1, dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    vcfc.encode_rows_device(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, total, out.data_ptr(), cap,
                            rec.data_ptr(), ws.data_ptr(), ws_bytes, err.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    e = int(err.cpu().numpy().view(np.uint64)[0])
    assert e == (2 << 8) | vcfc.E_TOOLONG
    r = rec.cpu().numpy()
    host = out[:int(r[2])].cpu().numpy().tobytes()
    assert host == G.oracle_encode_line(lines[0])[1] + G.oracle_encode_line(lines[1])[1]
