"""GPU parity for the sparse-file query (reference
query_sparse_file_fd, src/main.cpp:235-582): the sparse files are written by
this build's GPU sparsify; results byte-exact against the oracle restatement
and consistent with the reference CLI's own `main sparse-query` outputs
(tests/golden/sparse_query_cases.json), plus a chr22-shaped 2504-sample file
encoded on the GPU.  Through the C ABI (libvcfc.so) and the CLI (build/main)."""
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


@pytest.fixture(scope="module")
def ctx():
    import torch   # before libvcfc: one HIP runtime in the process
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import vcfc
    c = vcfc.Context(0)
    yield c
    c.close()


def gpu_sparsify(ctx, wd):
    def f(vcfc_bytes, path):
        src = path + ".vcfc"
        with open(src, "wb") as fh:
            fh.write(vcfc_bytes)
        ctx.sparsify_file(src, path)
        os.unlink(src)
    return f


def test_reference_cli_cases(ctx):
    d = G.sparse_query_cases()
    with tempfile.TemporaryDirectory(dir="/tmp") as wd:
        built = set()
        for c in d["cases"]:
            path = os.path.join(wd, c["file"] + ".sparse")
            if c["file"] not in built:
                G.build_sparse_file(d, c["file"], path, gpu_sparsify(ctx, wd))
                built.add(c["file"])
            st, out = ctx.sparse_query_status(path, c["query"].encode())
            assert G.check_sparse_case(c, st, out), (c, st, len(out))
            assert (st, out) == G.oracle_sparse_query(path, c["query"].encode()), c


def test_cli_sparse_query(ctx):
    main = os.path.join(REPO, "build", "main")
    d = G.sparse_query_cases()
    with tempfile.TemporaryDirectory(dir="/tmp") as wd:
        path = os.path.join(wd, "r.sparse")
        G.build_sparse_file(d, "random_100x10000", path, gpu_sparsify(ctx, wd))
        for c in d["cases"]:
            if c["file"] != "random_100x10000":
                continue
            r = subprocess.run([main, "sparse-query", path, c["query"]], capture_output=True, timeout=300)
            assert r.returncode == (0 if c["rc"] == 0 else 134), (c, r.stderr)
            assert G.check_sparse_case(c, 0 if c["rc"] == 0 else 8, r.stdout), c
        r = subprocess.run([main, "sparse-query", os.path.join(wd, "missing"), "1:1-2"], capture_output=True)
        assert r.returncode == 134


def test_chr22_shaped_2504_samples(ctx):
    """20k GPU-encoded chr22-shaped rows, sparsified on the GPU; ranges of
    every size against the oracle and against the rows themselves."""
    import torch
    import vcfc
    import workload
    n = 20000
    rows = workload.DeviceRows(torch, vcfc, n, 2504, 1, seed=21, device="cuda:0")
    body = rows.buf[:rows.total_bytes].cpu().numpy().tobytes()
    hdr = (b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT"
           + b"".join(b"\tS%d" % i for i in range(2504)) + b"\n")
    enc = ctx.compress_buffer(hdr + body)
    lines = body.split(b"\n")[:-1]
    pos = rows.pos
    with tempfile.TemporaryDirectory(dir="/tmp") as wd:
        src, sp = os.path.join(wd, "c.vcfc"), os.path.join(wd, "c.sparse")
        with open(src, "wb") as f:
            f.write(enc)
        ctx.sparsify_file(src, sp)
        for a, b in ((0, 0), (5, 6), (100, 2099), (0, n - 1), (19990, n - 1)):
            q = b"22:%d-%d" % (pos[a], pos[b])
            st, got = ctx.sparse_query_status(sp, q)
            want = b"".join(l + b"\n" for l in lines[a:b + 1])
            assert st == 0 and got == want, (a, b, st, len(got), len(want))
        for q in (b"22:%d-%d" % (pos[7] + 1, pos[9]), b"22:1-%d" % pos[3], b"21:%d-%d" % (pos[0], pos[50]),
                  b"22:%d-%d" % (pos[n - 1] + 5, pos[n - 1] + 9)):
            assert ctx.sparse_query_status(sp, q) == G.oracle_sparse_query(sp, q), q
