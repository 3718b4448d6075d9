"""Sharded sparsify (SURVEY §8 e) on CPU: world_size 2/3 over gloo run
dist_compress.sparsify_shards.  Each rank's shard step plans its records
with one halo record each side through k_sparse_plan on the CPU emulator (the
product kernel standing in for the GPU) and writes them as
vcfc_sparsify_shard does; the single-process fallback is the oracle's
sparsify.  The stitched sparse file must equal the reference's (hole-aware
digest), including the fallback cases (out-of-order POS, an unparsable POS)."""
import os
import struct
import sys
import tempfile

import pytest
import torch.multiprocessing as mp

import golden_io as G
import sparse_digest

sys.path.insert(0, os.path.join(G.REPO, "vcf-compression_amd"))
import dist_compress as D  # noqa: E402

NONE = (1 << 64) - 1


def _header_end(v):
    p = 0
    while v[p:p + 1] == b"#":
        p = v.index(b"\n", p) + 1
    return p


def _rec_index(body):
    ro, p = [], 0
    while len(body) - p >= 8:
        L = ((body[p] & 0x3F) << 24) | (body[p + 1] << 16) | (body[p + 2] << 8) | body[p + 3]
        ro.append(p)
        p += 8 + L - 4
    ro.append(p)
    return ro


def _emu_shard(in_path, out_path, rank, world):
    """vcfc_sparsify_shard's contract with the emulated plan kernel."""
    import emu_io as E
    v = open(in_path, "rb").read()
    h = _header_end(v)
    body = v[h:]
    rec = _rec_index(body)
    n = len(rec) - 1
    data_start = h + 8
    lo, hi = n * rank // world, n * (rank + 1) // world
    a, b = max(lo - 1, 0), min(hi + 1, n)
    err, anomaly, fo, pf = None, 0, [], b""
    if hi > lo:
        ro = [x - rec[a] for x in rec[a:b + 1]]
        fo, pf, st = E.emu_sparse_plan(body[rec[a]:rec[b]], ro, data_start)
        if st[0] != NONE:
            err = a + (int(st[0]) >> 8)
        anomaly = int(st[1] != 0)
    info = [lo, hi, err, anomaly]
    if out_path is None:
        return 0, info
    if err is not None or anomaly:
        return 5, info
    fd = os.open(out_path, os.O_WRONLY | os.O_CREAT, 0o600)
    if rank == 0:
        os.pwrite(fd, v[:h] + (b"\0" * 8 if n == 0 else b""), 0)
    for g in range(lo, hi):
        i = g - a
        if g == 0:
            os.pwrite(fd, struct.pack("<Q", int(fo[i]) - data_start), data_start - 8)
        os.pwrite(fd, bytes(pf[16 * i:16 * i + 16]) + body[rec[g]:rec[g + 1]], int(fo[i]))
    os.close(fd)
    return 0, info


def _oracle_whole(in_path, out_path):
    v = open(in_path, "rb").read()
    return G.oracle().vcfo_sparsify(v, len(v), out_path.encode())


def _worker(rank, world, port, in_path, out_path, q):
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(vals):
        out = [None] * world
        dist.all_gather_object(out, vals)
        return out
    st = D.sparsify_shards(rank, world, lambda w: _emu_shard(in_path, out_path if w else None, rank, world),
                           lambda: _oracle_whole(in_path, out_path), allgather)
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
            p.join(180)
            assert p.exitcode == 0
        res = sorted(q.get() for _ in range(world))
        want_st = G.oracle().vcfo_sparsify(v, len(v), rp.encode())
        return [r[1] for r in res], want_st, sparse_digest.digest(op), sparse_digest.digest(rp)


def _swap_records(v, i, j):
    h = _header_end(v)
    body = v[h:]
    rec = _rec_index(body)
    rs = [body[rec[k]:rec[k + 1]] for k in range(len(rec) - 1)]
    rs[i], rs[j] = rs[j], rs[i]
    return v[:h] + b"".join(rs)


def _break_pos(v, i):
    h = _header_end(v)
    body = bytearray(v[h:])
    rec = _rec_index(bytes(body))
    p = body.index(b"\t", rec[i] + 8) + 1   # first byte of POS
    body[p] = ord("x")
    return v[:h] + bytes(body)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_sparsify_equals_reference(world):
    v = G.gz("random_100x10000.vcfc.gz")
    sts, want_st, got, want = _run(world, v, 29600 + world)
    assert want_st == 0 and all(s == 0 for s in sts)
    assert got == want == G.manifest()["sparse_100x10000"]


def test_sharded_sparsify_fallbacks():
    v = G.gz("random_100x10000.vcfc.gz")
    # out-of-order POS across the shard boundary: rank 0 replays the whole file
    sts, want_st, got, want = _run(2, _swap_records(v, 49, 50), 29611)
    assert want_st == 0 and all(s == 0 for s in sts) and got == want
    # an unparsable POS in the second shard: the reference's partial file and status
    sts, want_st, got, want = _run(2, _break_pos(v, 70), 29612)
    assert want_st != 0 and all(s == want_st for s in sts) and got == want
    # the overlapping / duplicate-POS edge file
    sts, want_st, got, want = _run(2, G.gz("sparse_edge.vcfc.gz"), 29613)
    assert all(s == want_st for s in sts) and got == want == G.manifest()["sparse_edge"]
