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


def _oracle_range(in_path, off, length, fd, out_off):
    """vcfc.Context.compress_range with the oracle standing in for the GPU:
    (status, bytes written, failing line in the range, lines in the range)."""
    with open(in_path, "rb") as f:
        f.seek(off)
        buf = f.read(length)
    st, out, line = G.oracle_compress(buf)
    mv, o = memoryview(out), 0
    while o < len(out):
        o += os.pwrite(fd, mv[o:], out_off + o)
    lines = buf.count(b"\n") + (1 if buf and not buf.endswith(b"\n") else 0)
    return st, len(out), line, lines


class _MemHeld:
    """vcfc.Held stand-in: the oracle's output of a range, placed by pwrite."""

    def __init__(self, b):
        self.b = b

    def place(self, fd, off):
        mv, o = memoryview(self.b), 0
        while o < len(self.b):
            o += os.pwrite(fd, mv[o:], off + o)
        return 0

    def free(self):
        self.b = None


def _oracle_hold(in_path, off, length):
    """vcfc.Context.compress_range_held with the oracle standing in for the
    GPU: (status, bytes, failing line in the range, lines in the range, held)."""
    with open(in_path, "rb") as f:
        f.seek(off)
        buf = f.read(length)
    st, out, line = G.oracle_compress(buf)
    lines = buf.count(b"\n") + (1 if buf and not buf.endswith(b"\n") else 0)
    return st, len(out), line, lines, _MemHeld(out)


def _worker(rank, world, port, in_path, out_path, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(vals):
        out = [None] * world
        dist.all_gather_object(out, vals)
        return out
    st, total, line = D.compress_shard(in_path, out_path, rank, world, _oracle_range, _oracle_hold, allgather)
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


def test_rank_failure_travels_through_the_allgather():
    """A rank whose encoder raises (no GPU, I/O) reports E_IO through the
    all-gather instead of leaving the other ranks waiting; every rank returns
    the same status, and the output holds the ranks before it."""
    data = G.gz("random_100x10000.vcf.gz")
    with tempfile.TemporaryDirectory() as d:
        ip, op = os.path.join(d, "in.vcf"), os.path.join(d, "out.vcfc")
        with open(ip, "wb") as f:
            f.write(data)
        open(op, "wb").close()
        slots, calls = {}, {0: 0, 1: 0}

        def fake_gather(r):
            def g(vals):   # the k-th all-gather of rank r sees the k-th of the ranks before it
                k = calls[r]
                calls[r] += 1
                slots[(r, k)] = vals
                return [slots[(q, k)] for q in sorted(q for q, kk in slots if kk == k)]
            return g

        def boom(*a):
            raise RuntimeError("device lost")
        # run rank 0 with the oracle, then rank 1 failing (its all-gathers see
        # rank 0's values)
        r0 = D.compress_shard(ip, op, 0, 2, _oracle_range, _oracle_hold, fake_gather(0))
        r1 = D.compress_shard(ip, op, 1, 2, _oracle_range, boom, fake_gather(1))
        assert r1[0] == D.E_IO and r1[2] == -1
        pts = D.split_points(len(data), 2, lambda o, n: data[o:o + n])
        assert open(op, "rb").read() == G.oracle_compress(data[:pts[1]])[1]


def test_hold_bytes_is_a_share_of_the_host(monkeypatch):
    """The held-output bound: 3/4 of MemAvailable over the node's
    ranks less 1 GiB of pinned buffers each, capped by VCFC_HOLD_GB (32 GiB
    default), never below one 64 MiB block."""
    import vcfc
    G = 1 << 30
    monkeypatch.delenv("VCFC_HOLD_GB", raising=False)
    assert vcfc.hold_bytes(8, avail=256 * G) == 23 * G            # 192 GiB / 8 - 1
    assert vcfc.hold_bytes(1, avail=1024 * G) == 32 * G           # capped
    assert vcfc.hold_bytes(8, avail=4 * G) == 64 << 20            # floor
    monkeypatch.setenv("VCFC_HOLD_GB", "2")
    assert vcfc.hold_bytes(8, avail=256 * G) == 2 * G
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    monkeypatch.setenv("VCFC_HOLD_GB", "100")
    assert vcfc.hold_bytes(avail=64 * G) == 11 * G               # 48 GiB / 4 - 1
    assert vcfc.mem_available() is None or vcfc.mem_available() > 0


def test_held_releases_on_exit_and_gc():
    import vcfc
    freed = []

    class H(vcfc.Held):
        def free(self):
            freed.append(self._h)
            self._h = None
    with H(1234):
        pass
    h = H(99)
    del h
    assert freed == [1234, None, 99]


def _failing_worker(rank, world, port, mode):
    """One rank of a gloo job in which rank 1 fails before the data-path
    all-gather: `raise` (its setup raises, as an out-of-memory allocation
    would) or `die` (the process is gone, as after the OOM killer)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      VCFC_DIST_TIMEOUT_S="15")
    D.init_group(dist, "gloo")

    def allgather(vals):
        out = [None] * world
        dist.all_gather_object(out, vals)
        return out

    def setup():
        if rank == 1 and mode == "raise":
            raise MemoryError("HBM allocation failed")
        if rank == 1 and mode == "die":
            os._exit(3)
        return 7
    try:
        assert D.setup_all_or_none(rank, allgather, setup) == 7
        allgather([1])   # the all-gather of shard sizes
        code = 0
    except D.RankFailed:
        code = 11
    except Exception:   # the backend's error for a peer that is gone
        code = 12
    sys.stdout.flush()
    os._exit(code)


@pytest.mark.parametrize("mode", ["raise", "die"])
def test_rank_failing_before_the_allgather_ends_every_rank(mode):
    """a rank that fails before the all-gather must make
    the others exit non-zero within the collectives' timeout (here 15 s),
    never hang.  A raising rank reports through the status all-gather (every
    rank raises RankFailed); a dead rank surfaces as the backend's error."""
    import time
    ctx = mp.get_context("spawn")
    port = 29530 + (mode == "die")
    t0 = time.time()
    ps = [ctx.Process(target=_failing_worker, args=(r, 2, port, mode)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(90)
    dt = time.time() - t0
    alive = [p for p in ps if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "a rank was still waiting after 90 s"
    # exit codes: 11 = RankFailed, 12 = the backend's error, 3 = the dead rank
    if mode == "raise":
        assert [p.exitcode for p in ps] == [11, 11]
    else:
        assert ps[1].exitcode == 3 and ps[0].exitcode in (11, 12)
    assert dt < 75
