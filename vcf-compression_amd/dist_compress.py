"""Multi-GPU `compress` (SURVEY §8 e): one process per GPU, rows sharded as
contiguous line-aligned byte ranges of the input file, one all-gather of the
per-shard output sizes to stitch the output.

compress() (reference src/compress.cpp:205-257) is stateless per line -- the
schema it tracks is never read by the encoder -- so any split at a line
boundary can be compressed independently and the outputs concatenated in
order.  Each rank encodes its slice on its own GPU (vcfc.Context.compress_buffer),
all-gathers the byte counts (RCCL on GPU ranks, gloo in the CPU tests), and
pwrites its bytes at the exclusive prefix.

Run: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
         vcf-compression_amd/dist_compress.py [sparsify] in out

`sparsify` shards sparsify_file the same way (records split evenly, one
halo record each side, one all-gather of the plans' verdicts).
"""
import os
import sys


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


def compress_shard(in_path, out_path, rank, world, encode, allgather):
    """encode(bytes) -> (status, out_bytes, err_line_in_slice), where on a
    failing line out_bytes holds the output of the slice's lines before it;
    allgather(list_of_ints_local) -> list of per-rank lists.
    Returns (status, total_bytes, global_err_line).  The output file equals
    the single-process output: on a failure, everything before the first
    failing line in file order (the reference stops there)."""
    size = os.path.getsize(in_path)
    with open(in_path, "rb") as f:
        def read_at(off, n):
            f.seek(off)
            return f.read(n)
        pts = split_points(size, world, read_at)
        f.seek(pts[rank])
        mine = f.read(pts[rank + 1] - pts[rank])
        # lines before my slice (for global line numbers of errors)
        f.seek(0)
        lines_before = 0
        left = pts[rank]
        while left > 0:
            b = f.read(min(left, 1 << 24))
            lines_before += b.count(b"\n")
            left -= len(b)
    st, out, err_line = encode(mine)
    g = allgather([len(out), st, (lines_before + err_line) if st else -1])
    # the first failing rank (shards are in file order) holds the first
    # failing line: it writes its partial output, later ranks write nothing
    first_bad = next((r for r, x in enumerate(g) if x[1] != 0), world)
    counts = [x[0] if r <= first_bad else 0 for r, x in enumerate(g)]
    offs, total = exclusive_offsets(counts)
    status, gline = (g[first_bad][1], g[first_bad][2]) if first_bad < world else (0, -1)
    fd = os.open(out_path, os.O_WRONLY | os.O_CREAT, 0o644)
    try:
        if out and rank <= first_bad:
            os.pwrite(fd, out, offs[rank])
        if rank == world - 1:
            os.ftruncate(fd, total)
    finally:
        os.close(fd)
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
        dist.init_process_group("nccl", device_id=dev)
    if rank == 0:
        open(out_path, "wb").close()
    if world > 1:
        dist.barrier()
    ctx = vcfc.Context(local)

    def encode(buf):
        st, out, line = ctx.compress_status(buf)
        if st not in (vcfc.OK, vcfc.E_LT8COLS, vcfc.E_8COLS, vcfc.E_HEADER):
            vcfc.raise_for(st)
        return st, out, line

    def allgather(vals):
        if world == 1:
            return [vals]
        t = torch.tensor(vals, dtype=torch.int64, device=dev)
        out = torch.empty(world * len(vals), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(out, t)   # RCCL over xGMI
        return out.view(world, len(vals)).cpu().tolist()

    if mode == "sparsify":
        st = sparsify_shards(rank, world,
                             lambda write: ctx.sparsify_shard(in_path, out_path if write else None, rank, world),
                             lambda: ctx.sparsify_status(in_path, out_path), allgather)
        line = -1
    else:
        st, total, line = compress_shard(in_path, out_path, rank, world, encode, allgather)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and st:
        print("vcfc: %s (input line %d)" % (vcfc.strerror(st), line), file=sys.stderr)
    sys.exit(1 if st else 0)


if __name__ == "__main__":
    main()
