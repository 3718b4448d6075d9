"""GPU: sharded sparsify through the C ABI (vcfc_sparsify_shard, SURVEY §8 e)
with 1/2/3 ranks, all on cuda:0 (one process per rank, gloo for the
all-gather: RCCL refuses two ranks on one device).  The stitched sparse file
equals the reference's (hole-aware digest of its `main sparsify` output) and
the single-process fallback covers out-of-order POS and unparsable records."""
import os
import sys
import tempfile

import pytest
import torch.multiprocessing as mp

import golden_io as G
import sparse_digest
import test_shard_sparse as T

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(G.REPO, "vcf-compression_amd"))


def _worker(rank, world, port, in_path, out_path, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(G.REPO, "vcf-compression_amd"))
    import dist_compress as D
    import vcfc
    assert torch.cuda.is_available()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = vcfc.Context(0)

    def allgather(vals):
        out = [None] * world
        dist.all_gather_object(out, vals)
        return out
    st = D.sparsify_shards(rank, world,
                           lambda w: ctx.sparsify_shard(in_path, out_path if w else None, rank, world),
                           lambda: ctx.sparsify_status(in_path, out_path), allgather)
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, st))


def _run(world, v, port):
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        ip, op, rp = os.path.join(d, "in.vcfc"), os.path.join(d, "out.sparse"), os.path.join(d, "ref.sparse")
        with open(ip, "wb") as f:
            f.write(v)
        open(op, "wb").close()
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=_worker, args=(r, world, port, ip, op, q)) for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(120)
            assert p.exitcode == 0
        sts = [r[1] for r in sorted(q.get() for _ in range(world))]
        want_st = G.oracle().vcfo_sparsify(v, len(v), rp.encode())
        return sts, want_st, sparse_digest.digest(op), sparse_digest.digest(rp)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_gpu_sharded_sparsify(world):
    v = G.gz("random_100x10000.vcfc.gz")
    sts, want_st, got, want = _run(world, v, 29700 + world)
    assert want_st == 0 and sts == [0] * world
    assert got == want == G.manifest()["sparse_100x10000"]


def test_gpu_sharded_sparsify_fallbacks():
    v = G.gz("random_100x10000.vcfc.gz")
    sts, want_st, got, want = _run(2, T._swap_records(v, 49, 50), 29711)
    assert want_st == 0 and sts == [0, 0] and got == want
    sts, want_st, got, want = _run(2, T._break_pos(v, 70), 29712)
    assert want_st != 0 and all(s != 0 for s in sts) and got == want
    sts, want_st, got, want = _run(2, G.gz("sparse_edge.vcfc.gz"), 29713)
    assert sts == [0, 0] and got == want == G.manifest()["sparse_edge"]
