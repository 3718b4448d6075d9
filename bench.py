#!/usr/bin/env python3
"""bench.py -- BASELINE.json's headline metric on MI355X.

metric : input GT bytes/sec encoded, 2504-sample x 1M-variant VCF (BASELINE
         configs[1], chr22-shaped synthetic rows generated in HBM).
step   : one pass of the hot path (reference compress_data_line,
         src/compress.cpp:5-203) over the whole batch resident in HBM:
         slot scan -> k_encode -> size scan -> k_compact, plus -- for N > 1
         -- one RCCL all-gather of the per-shard record byte counts (the
         stitch offsets of the output file).
scaling: weak.  Every rank encodes its own 1M-row shard (rows are
         independent; the shards are contiguous row ranges of one file).
value  : GT bytes of all ranks / (max over ranks of the timed wall time).

Also printed: `roofline` for the dominant kernel k_encode (algorithmic bytes
= line bytes read + record bytes written, per launch / its HIP-event time)
and `cpu_baseline`: the reference's own `main compress` (oracle/_ref/main,
compiled from the reference sources; single-threaded) on a bounded sample of
the same rows, timed on this host.

Run: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RCCL).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "vcf-compression_amd"))
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=1_000_000, help="rows per GPU")
    ap.add_argument("--samples", type=int, default=2504)
    ap.add_argument("--law", type=int, default=1, help="1 = chr22-shaped (headline), 0 = random_vcf law")
    ap.add_argument("--cpu-rows", type=int, default=120_000, help="rows in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify-rows", type=int, default=64, help="rows checked against the CPU path")
    ap.add_argument("--mode", choices=["encode", "decode"], default="encode",
                    help="encode = the headline (BASELINE metric); decode = row f1 (config 5 building block)")
    return ap.parse_args()


def cpu_baseline(rows, torch, args):
    """Time the reference CLI (or, if absent, the C restatement) on the first
    --cpu-rows rows of the benchmark shard; return (dict, sample_out_bytes)."""
    import numpy as np
    k = min(args.cpu_rows, rows.n)
    lo = rows.line_off[:k + 1].cpu().numpy() if k < rows.n else None
    end = int(lo[k]) if lo is not None else rows.total_bytes
    body = rows.buf[:end].cpu().numpy().tobytes()
    header = ("##fileformat=VCFv4.2\n##source=vcfc-mi355x bench\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT"
              + "".join("\tS%d" % i for i in range(rows.samples)) + "\n").encode()
    gt = 4 * rows.samples * k
    ref = os.path.join(REPO, "oracle", "_ref", "main")
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        src, dst = os.path.join(d, "s.vcf"), os.path.join(d, "s.vcfc")
        with open(src, "wb") as f:
            f.write(header + body)
        if os.path.exists(ref):
            t0 = time.perf_counter()
            r = subprocess.run([ref, "compress", src, dst], capture_output=True)
            dt = time.perf_counter() - t0
            if r.returncode != 0:
                raise RuntimeError("reference compress failed: %s" % r.stderr[-400:])
            kind = "reference"
            out = open(dst, "rb").read()[len(header):]
        else:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            import golden_io as G
            t0 = time.perf_counter()
            st, out, _ = G.oracle_compress(header + body)
            dt = time.perf_counter() - t0
            assert st == 0
            out = out[len(header):]
            kind = "port"
    return ({"value": round(gt / dt / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": kind,
             "sample": "first %d rows of the rank-0 shard (%d GT bytes, %.1f MB file), `main compress` wall time %.2f s"
                       % (k, gt, (len(header) + len(body)) / 1e6, dt)}, out, k)


def load_pmc(workload_key):
    p = os.path.join(REPO, "profiles", "pmc_k_encode.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        if d.get("workload") == workload_key:
            return d.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


def bench_decode(args, torch, vcfc, workload):
    """Row f1: decode the same synthetic batch (device-resident records made
    by the GPU encoder) back to VCF lines; every output byte is checked
    against the original rows on the GPU.  One GPU (replicas only)."""
    import numpy as np
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n, S = args.rows, args.samples
    rows = workload.DeviceRows(torch, vcfc, n, S, args.law, seed=1000, device=dev)
    ws_bytes = vcfc.workspace_size(n, rows.line_bytes)
    cap = vcfc.encode_bound(n, rows.line_bytes)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    recs = torch.empty(cap, dtype=torch.uint8, device=dev)
    rec = torch.empty(n + 1, dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    vcfc.encode_rows_device(rows.buf.data_ptr(), rows.line_off.data_ptr(), rows.line_len.data_ptr(), n,
                            rows.line_bytes, recs.data_ptr(), cap, rec.data_ptr(), ws.data_ptr(), ws_bytes,
                            err.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    rec_bytes = int(rec[n].item())
    del ws
    dws_bytes = vcfc.decode_workspace_size(n)
    dws = torch.empty(dws_bytes, dtype=torch.uint8, device=dev)
    out_cap = rows.total_bytes + 64
    out = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    loff = torch.empty(n + 1, dtype=torch.int64, device=dev)

    def step():
        vcfc.decode_records_device(recs.data_ptr(), rec_bytes, rec.data_ptr(), n, S, out.data_ptr(), out_cap,
                                   loff.data_ptr(), dws.data_ptr(), dws_bytes, err.data_ptr(), stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        step()
    e1.record()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    ev_ms = e0.elapsed_time(e1) / args.steps
    e = int(err.cpu().numpy().view(np.uint64)[0])
    total = int(loff[n].item())
    # (light plan: a code-4 report would mean "rerun exact"; it is counted as a failure here)
    identical = e == vcfc.NO_ERROR and total == rows.total_bytes and bool(torch.equal(out[:total], rows.buf[:total]))
    alg = rec_bytes + total
    res = {"metric": "decoded GT bytes/sec, 2504-sample x 1M-variant .vcfc (row f1)",
           "value": round(rows.gt_bytes * args.steps / elapsed / 1e9, 2), "unit": "GB/s", "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
           "higher_is_better": True, "scaling": "replicas", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (generated and encoded in HBM)",
           "config": {"workload": "%s %d samples x %d variants" % ("chr22-shaped" if args.law == 1 else
                                                                   "random_vcf-law", S, n),
                      "record_bytes": rec_bytes, "line_bytes": total},
           "roofline": {"kernel": "k_dec_plan + k_dec_write", "bound": "hbm",
                        "achieved": round(alg / (ev_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / (ev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                        "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(ev_ms, 4)},
           "output_identical_to_input_rows": identical}
    print(json.dumps(res), flush=True)


def main():
    args = parse()
    if args.mode == "decode":
        import torch
        import vcfc
        import workload
        return bench_decode(args, torch, vcfc, workload)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch          # before libvcfc: one HIP runtime per process
    import torch.distributed as dist
    import vcfc
    import workload

    dev = torch.device("cuda:%d" % local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    n, S = args.rows, args.samples
    rows = workload.DeviceRows(torch, vcfc, n, S, args.law, seed=1000 + rank, device=dev, row0=rank * n)
    ws_bytes = vcfc.workspace_size(n, rows.line_bytes)
    cap = vcfc.encode_bound(n, rows.line_bytes)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    rec = torch.empty(n + 1, dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    timer = vcfc.StageTimer()
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step(timed):
        f = timer.encode if timed else vcfc.encode_rows_device
        f(rows.buf.data_ptr(), rows.line_off.data_ptr(), rows.line_len.data_ptr(), n, rows.line_bytes,
          out.data_ptr(), cap, rec.data_ptr(), ws.data_ptr(), ws_bytes, err.data_ptr(), stream)
        if world > 1:
            # stitch: every rank learns every shard's record bytes -> its file offset
            dist.all_gather_into_tensor(counts, rec[n:n + 1])

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    stages, calls = timer.read()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    e = int(err.cpu().numpy().view(np.uint64)[0])
    if e != vcfc.NO_ERROR:
        raise RuntimeError("encode reported row error %x" % e)
    out_bytes = int(rec[n].item())
    ms_step = elapsed * 1e3 / args.steps
    gt_total = rows.gt_bytes * world
    value = gt_total * args.steps / elapsed / 1e9
    k_ms = stages["k_encode"] / max(calls, 1)
    alg = rows.line_bytes + out_bytes
    wl = "chr22-shaped" if args.law == 1 else "random_vcf-law"
    wkey = "%s/%dx%d" % (wl, S, n)
    roof = {"kernel": "k_encode", "bound": "hbm", "achieved": round(alg / (k_ms * 1e-3) / 1e9, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": load_pmc(wkey),
            "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(k_ms, 4),
            "stages_ms": {k: round(v / max(calls, 1), 4) for k, v in stages.items()}}
    res = {"metric": "input GT bytes/sec encoded, 2504-sample x 1M-variant VCF",
           "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic (generated in HBM)",
           "config": {"workload": "%s %d samples x %d variants per GPU (BASELINE configs[1])" % (wl, S, n),
                      "samples": S, "rows_per_gpu": n, "gt_bytes_per_gpu": rows.gt_bytes,
                      "line_bytes_per_gpu": rows.line_bytes, "record_bytes_per_gpu": out_bytes,
                      "compression_ratio": round(out_bytes / rows.line_bytes, 4),
                      "parallelism": "row shards x%d, RCCL all-gather of shard sizes" % world},
           "roofline": roof}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, cpu_out, k = cpu_baseline(rows, torch, args)
        res["cpu_baseline"] = cb
        gpu_out = out[:int(rec[k].item())].cpu().numpy().tobytes()
        res["cpu_baseline"]["gpu_output_identical"] = gpu_out == cpu_out
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
