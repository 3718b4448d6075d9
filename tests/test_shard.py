"""Multi-rank stitch logic (SURVEY §8 e) on CPU: world_size 1/2/4 with the
gloo backend; each rank encodes its line-aligned slice (the oracle stands in
for the GPU encoder here) and the stitched output must equal the single-rank
output and the reference's golden bytes."""
import os
import sys
import tempfile

import pytest
import torch.multiprocessing as mp

import golden_io as G

sys.path.insert(0, os.path.join(G.REPO, "vcf-compression_amd"))
import dist_compress as D  # noqa: E402


def _oracle_encode(buf):
    st, out, line = G.oracle_compress(buf)
    return st, out, line


def _worker(rank, world, port, in_path, out_path, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(vals):
        out = [None] * world
        dist.all_gather_object(out, vals)
        return out
    st, total, line = D.compress_shard(in_path, out_path, rank, world, _oracle_encode, allgather)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, st, total, line))


def _run(world, data, port):
    with tempfile.TemporaryDirectory() as d:
        ip, op = os.path.join(d, "in.vcf"), os.path.join(d, "out.vcfc")
        with open(ip, "wb") as f:
            f.write(data)
        open(op, "wb").close()
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=_worker, args=(r, world, port, ip, op, q)) for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(120)
            assert p.exitcode == 0
        res = sorted(q.get() for _ in range(world))
        return res, open(op, "rb").read()


def test_split_points_line_aligned():
    data = G.gz("fuzz_encode.vcf.gz")
    for world in (1, 2, 3, 8, 64):
        pts = D.split_points(len(data), world, lambda o, n: data[o:o + n])
        assert pts[0] == 0 and pts[-1] == len(data) and pts == sorted(pts)
        assert all(p == 0 or p == len(data) or data[p - 1:p] == b"\n" for p in pts)


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_stitch_equals_reference(world):
    data = G.gz("random_100x10000.vcf.gz")
    res, out = _run(world, data, 29500 + world)
    assert all(r[1] == 0 for r in res)
    assert out == G.gz("random_100x10000.vcfc.gz")


def test_gloo_stitch_fuzz_and_error_line():
    data = G.gz("fuzz_encode.vcf.gz")
    res, out = _run(2, data, 29507)
    assert out == G.gz("fuzz_encode.vcfc.gz")
    # a bad line in the second half: status + global line number agree with
    # the single-process oracle
    lines = data.split(b"\n")
    k = len(lines) * 3 // 4
    lines[k] = b"1\t2\t3"
    bad = b"\n".join(lines)
    st1, out1, line1 = G.oracle_compress(bad)
    res, out = _run(2, bad, 29508)
    assert st1 == 1 and all(r[1] == 1 and r[3] == line1 for r in res)
    assert out == out1   # everything before the failing line, as one process writes it
    # failing line in the first shard: the second shard writes nothing
    lines = data.split(b"\n")
    lines[len(lines) // 5] = b"1\t2\t3"
    bad = b"\n".join(lines)
    st1, out1, line1 = G.oracle_compress(bad)
    res, out = _run(2, bad, 29509)
    assert st1 == 1 and all(r[1] == 1 and r[3] == line1 for r in res) and out == out1
