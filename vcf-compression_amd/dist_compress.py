"""Multi-GPU `compress` (SURVEY §8 e): one process per GPU, rows sharded as
contiguous line-aligned byte ranges of the input file, one all-gather of the
per-shard output sizes to stitch the output.

compress() (reference src/compress.cpp:205-257) is stateless per line -- the
schema it tracks is never read by the encoder -- so any split at a line
boundary can be compressed independently and the outputs concatenated in
order.  Each rank streams its slice through the ingest pipeline on its own GPU
(reader threads, pinned H2D, GPU line index + encode): rank 0 writes its
output in place, every other rank holds its output in host memory
(vcfc.Context.compress_range_held); one all-gather of (bytes, status, failing
line, lines) -- RCCL on GPU ranks, gloo in the CPU tests -- gives each rank
its offset, the exclusive prefix of the byte counts, where it writes the held
bytes once.

Run: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
         vcf-compression_amd/dist_compress.py [sparsify] in out

`sparsify` shards sparsify_file the same way (records split evenly, one
halo record each side, one all-gather of the plans' verdicts).
"""
import os
import sys

E_IO = 7   # include/vcfc.h VCFC_E_IO
# Bound on every collective (init, all-gather, barrier): a rank that dies
# before a collective must not leave its peers waiting for the backend's
# default (about 10 minutes for NCCL), past a driver's run limit.
DIST_TIMEOUT_S = 120


class RankFailed(RuntimeError):
    """Raised on every rank when some rank's setup failed (setup_all_or_none)."""


def dist_timeout():
    """The collectives' timeout (timedelta): VCFC_DIST_TIMEOUT_S, default 120 s."""
    from datetime import timedelta
    return timedelta(seconds=float(os.environ.get("VCFC_DIST_TIMEOUT_S", DIST_TIMEOUT_S)))


def init_group(dist, backend, device_id=None):
    """dist.init_process_group with the bounded timeout (and the rank's device
    for RCCL), so a missing or dead peer ends the job with an error instead of
    a hang."""
    kw = {"timeout": dist_timeout()}
    if device_id is not None:
        kw["device_id"] = device_id
    dist.init_process_group(backend, **kw)


def setup_all_or_none(rank, allgather, fn):
    """Run this rank's setup fn() (allocations, input generation) and put its
    outcome through one all-gather before any data-path collective: if any
    rank failed, every rank raises RankFailed naming the failed ranks (the
    failing rank chains its own exception), so all exit non-zero together
    instead of the healthy ranks waiting in a later collective for a rank
    that is gone.  Returns fn()'s value."""
    err, val = None, None
    try:
        val = fn()
    except Exception as e:   # reported through the all-gather
        err = e
        print("vcfc rank %d: setup failed: %r" % (rank, e), file=sys.stderr, flush=True)
    g = allgather([0 if err is None else 1])
    bad = [r for r, x in enumerate(g) if x[0]]
    if bad:
        raise RankFailed("setup failed on rank(s) %s" % bad) from err
    return val
# Output a rank holds in host memory until its offset is known (the rest
# spills to a temporary file beside the output): vcfc.hold_bytes(), this
# rank's share of the host's MemAvailable, capped by VCFC_HOLD_GB (32 GiB).


def split_points(data_len, world, read_at):
    """Line-aligned split offsets [0 = p0 <= p1 <= ... <= pN = data_len].
    read_at(off, n) -> bytes; a split moves forward to just after a '\\n'."""
    pts = [0]
    for k in range(1, world):
        p = max(data_len * k // world, pts[-1])
        while p < data_len:
            chunk = read_at(p, 1 << 16)
            i = chunk.find(b"\n")
            if i >= 0:
                p += i + 1
                break
            p += len(chunk)
        pts.append(min(p, data_len))
    pts.append(data_len)
    return pts


def exclusive_offsets(counts):
    offs, acc = [], 0
    for c in counts:
        offs.append(acc)
        acc += c
    return offs, acc


def compress_shard(in_path, out_path, rank, world, compress_range, hold, allgather):
    """One rank of a sharded compress.

    compress_range(in_path, off, length, fd, out_off) -> (status, bytes
    written, 1-based failing line in the range or -1, lines in the range)
    streams a line-aligned byte range through the ingest pipeline
    (vcfc.Context.compress_range) straight into fd at out_off: rank 0, whose
    output starts the file, uses it.  hold(in_path, off, length) -> (status,
    bytes, failing line, lines, held) does the same with the output held in
    host memory (spilling past a bound, vcfc_compress_range_held): every
    other rank uses it, and once one all-gather of (bytes, status, failing
    line, lines) has given it its offset -- the exclusive prefix of the byte
    counts -- places the held bytes there with held.place(fd, off).  Output
    that fits in memory is written once, to its final place; no rank reads
    outside its own range.  A second all-gather carries the placements'
    statuses.  allgather(list_of_ints) -> per-rank lists.

    Returns (status, total bytes, global failing line or -1) -- the same on
    every rank.  The output file equals the single-process output: on a
    failure, everything before the first failing line in file order (the
    reference stops there, src/compress.cpp:205-257).  Errors that are not
    about the VCF (HIP, I/O) travel through the same all-gathers, so no rank
    is left waiting in a collective."""
    size = os.path.getsize(in_path)
    with open(in_path, "rb") as f:
        def read_at(off, n):
            f.seek(off)
            return f.read(n)
        pts = split_points(size, world, read_at)
    lo, hi = pts[rank], pts[rank + 1]
    fd = os.open(out_path, os.O_WRONLY | os.O_CREAT, 0o644)
    held = None
    try:
        try:
            if rank == 0:
                st, nb, eline, lines = compress_range(in_path, lo, hi - lo, fd, 0)
            else:
                st, nb, eline, lines, held = hold(in_path, lo, hi - lo)
        except Exception as e:   # still take part in the collectives
            print("vcfc rank %d: %s" % (rank, e), file=sys.stderr)
            st, nb, eline, lines = E_IO, 0, -1, 0
        g = allgather([int(nb), int(st), int(eline), int(lines)])
        # the first failing rank (shards are in file order) holds the first
        # failing line: it places its partial output, later ranks nothing
        first_bad = next((r for r, x in enumerate(g) if x[1] != 0), world)
        counts = [x[0] if r <= first_bad else 0 for r, x in enumerate(g)]
        offs, total = exclusive_offsets(counts)
        if first_bad < world:
            status = g[first_bad][1]
            eb = g[first_bad][2]
            gline = sum(x[3] for x in g[:first_bad]) + eb if eb >= 0 else -1
        else:
            status, gline = 0, -1
        pst = 0
        try:
            if rank > 0 and rank <= first_bad and counts[rank]:
                pst = held.place(fd, offs[rank]) if held is not None else E_IO
            if rank == world - 1:
                os.ftruncate(fd, total)
        except Exception as e:
            print("vcfc rank %d: %s" % (rank, e), file=sys.stderr)
            pst = E_IO
        p = allgather([int(pst)])
        if any(x[0] for x in p) and status == 0:
            status = next(x[0] for x in p if x[0])
    finally:
        os.close(fd)
        if held is not None:
            held.free()
    return status, total, gline


def sparsify_shards(rank, world, shard, whole, allgather):
    """Sharded sparsify_file (reference src/sparse.cpp:290-580; SURVEY §8 e).

    shard(write) -> (status, [lo, hi, first_err or None, anomaly]) plans this
    rank's records [lo, hi) with one halo record each side and, when write is
    true, writes them into the (already created) output; whole() -> status of
    the single-process sparsify, which replays the reference's write order;
    allgather(list_of_ints) -> per-rank lists.

    Every rank plans; one all-gather of (status, first unparsable record,
    anomaly) decides.  Clean everywhere: records sit at strictly increasing,
    disjoint offsets, so the ranks write their slices concurrently and the
    file equals the reference's sequential one.  Otherwise (out-of-order or
    overlapping POS, a record the reference throws on) rank 0 alone runs the
    replay.  Returns the job status (the same on every rank)."""
    st, info = shard(False)
    g = allgather([st, -1 if info[2] is None else int(info[2]), int(info[3])])
    if any(x[0] for x in g):
        return next(x[0] for x in g if x[0])
    if all(x[1] == -1 and x[2] == 0 for x in g):
        st, _ = shard(True)
    else:
        st = whole() if rank == 0 else 0
    g = allgather([st])
    return next((x[0] for x in g if x[0]), 0)


def main():
    import torch  # noqa: F401  (torch first: one HIP runtime)
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import vcfc
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    mode = "compress"
    if sys.argv[1] == "sparsify":
        mode = "sparsify"
        del sys.argv[1]
    in_path, out_path = sys.argv[1], sys.argv[2]
    dev = torch.device("cuda:%d" % local)
    torch.cuda.set_device(dev)
    if world > 1:
        init_group(dist, "nccl", device_id=dev)
    if rank == 0:
        open(out_path, "wb").close()
    if world > 1:
        dist.barrier()
    try:
        ctx = vcfc.Context(local)
    except RuntimeError as e:   # reported through the all-gather below
        print("vcfc rank %d: %s" % (rank, e), file=sys.stderr)
        ctx = None

    def compress_range(path, off, length, fd, out_off):
        if ctx is None:
            return vcfc.E_HIP, 0, -1, 0
        return ctx.compress_range(path, off, length, fd, out_off)

    def hold(path, off, length):
        if ctx is None:
            return vcfc.E_HIP, 0, -1, 0, None
        return ctx.compress_range_held(path, off, length, mem_bound=vcfc.hold_bytes(),
                                       spill_dir=os.path.dirname(os.path.abspath(out_path)))

    def allgather(vals):
        if world == 1:
            return [vals]
        t = torch.tensor(vals, dtype=torch.int64, device=dev)
        out = torch.empty(world * len(vals), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(out, t)   # RCCL over xGMI
        return out.view(world, len(vals)).cpu().tolist()

    if mode == "sparsify":
        # (a rank without a context reports E_HIP through the all-gathers
        # instead of raising before them: the other ranks would wait forever)
        def shard(write):
            if ctx is None:
                return vcfc.E_HIP, [0, 0, None, 0]
            return ctx.sparsify_shard(in_path, out_path if write else None, rank, world)

        def whole():
            return vcfc.E_HIP if ctx is None else ctx.sparsify_status(in_path, out_path)

        st = sparsify_shards(rank, world, shard, whole, allgather)
        line = -1
    else:
        st, total, line = compress_shard(in_path, out_path, rank, world, compress_range, hold, allgather)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and st:
        print("vcfc: %s (input line %d)" % (vcfc.strerror(st), line), file=sys.stderr)
    sys.exit(1 if st else 0)


if __name__ == "__main__":
    main()
