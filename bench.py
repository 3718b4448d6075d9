#!/usr/bin/env python3
"""bench.py -- BASELINE.json's headline metric on MI355X.

metric : input GT bytes/sec encoded, 2504-sample x 1M-variant VCF (BASELINE
         configs[1], chr22-shaped synthetic rows generated in HBM).
step   : one pass of the hot path (reference compress_data_line,
         src/compress.cpp:5-203) over the whole batch resident in HBM:
         slot scan -> k_encode -> size scan -> k_compact, plus -- for N > 1
         -- one RCCL all-gather of the per-shard record byte counts (the
         stitch offsets of the output file).
scaling: weak (default).  Every rank encodes its own 1M-row shard (rows are
         independent; the shards are contiguous row ranges of one file).
         With --gpus N > 1 the same process group then also times the
         strong split of the N=1 line's own 1M-row dataset (1M/N rows per
         rank, byte-identical slices) and reports it as the line's `strong`
         object -- BASELINE's fixed-dataset 1/2/4/8-GPU curve.
         --scaling strong: only the strong split (1M/N rows each).
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
    ap.add_argument("--rows", type=int, default=None, help="rows per GPU (default 1M; 100k in --mode biobank)")
    ap.add_argument("--samples", type=int, default=None, help="samples (default 2504; 100k in --mode biobank)")
    ap.add_argument("--law", type=int, default=1, choices=[0, 1, 2, 3],
                    help="1 = chr22-shaped (headline), 0 = random_vcf law, 2 = general shapes (SURVEY D3), "
                         "3 = alternating classes (SURVEY D3, the RLE worst case)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: every rank encodes --rows rows (with --gpus N > 1 the line also carries the "
                         "strong split of the N=1 dataset as its 'strong' object); strong: the --rows rows are "
                         "split over the ranks")
    ap.add_argument("--no-strong", action="store_true",
                    help="--gpus N > 1, weak scaling: skip the strong-split sub-measurement")
    ap.add_argument("--cpu-rows", type=int, default=None,
                    help="rows in the CPU-baseline sample (default: about 1.2 GB of lines)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify-rows", type=int, default=64, help="rows checked against the CPU path")
    ap.add_argument("--mode", choices=["encode", "biobank", "decode", "query", "ingest", "devfile", "sparse",
                                       "distfile"],
                    default="encode",
                    help="encode = the headline (BASELINE metric, configs[1]); biobank = configs[3] "
                         "(100k samples, one 100k-row batch of a 5M-row shard per GPU); decode = row f1; "
                         "query = row f2; ingest = row f4 (end-to-end file compress, configs[2]); "
                         "devfile = compress() of the configs[1] file already in HBM (line index + encode); "
                         "sparse = rows a7-a9 + f3 (sparsify, sparse-file query); distfile = the sharded "
                         "file -> file compress (row e: every rank its byte range, outputs held and placed at "
                         "the all-gathered offsets), --ingest-rows rows per rank")
    ap.add_argument("--dist-dir", default="/tmp/vcfc_distfile", help="--mode distfile: where the files go")
    ap.add_argument("--deferred-records", choices=["on", "off"], default="on",
                    help="devfile: vcfc_ctx_set_deferred_records (on by default since round 5: GT:DP:GQ-like rows "
                         "written straight to the output)")
    ap.add_argument("--line-index", choices=["hop", "scan"], default="hop",
                    help="--mode devfile: the line index (hop: line ends guessed from the header's sample count "
                         "and checked; scan: every byte)")
    ap.add_argument("--dev-chunk", type=int, default=0,
                    help="--mode devfile: chunk bytes of the device-resident compress (0: the whole file)")
    ap.add_argument("--rows-total", type=int, default=None,
                    help="--mode biobank: encode the rank's whole share of this many rows (5M = configs[3]) "
                         "as back-to-back --rows batches, every record digested and sampled rows re-encoded "
                         "by the CPU checker; a step is the whole shard")
    ap.add_argument("--sample-rows", type=int, default=1100,
                    help="--mode biobank --rows-total: random rows of every other batch digest-checked against "
                         "the oracle per pass (besides one whole batch per pass): 49 x 1100 + 100k > 150k rows per pass")
    ap.add_argument("--sparse-rows", type=int, default=200_000, help="rows of the --mode sparse file")
    ap.add_argument("--ingest-rows", type=int, default=200_000, help="rows of the --mode ingest file")
    ap.add_argument("--query-frac", type=float, default=0.125, help="rows selected by the --mode query range")
    a = ap.parse_args()
    big = a.mode == "biobank"
    if a.samples is None:
        a.samples = 100_000 if big else 2504
    if a.rows is None:
        a.rows = 100_000 if big else 1_000_000
    if a.cpu_rows is None:
        a.cpu_rows = max(1, int(2.4e9 // (4 * a.samples + 180)))   # ~235k rows at 2504 samples (~15 s, 1 core)
    return a


def law_name(law):
    return {0: "random_vcf-law", 1: "chr22-shaped", 2: "general-shapes (chrX haploid/GT:DP:GQ/missing)",
            3: "alternating-classes (every token a run / het 1/2)"}[law]


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
        par = None
        if kind == "reference":
            # the same sample over P processes (byte-balanced row shards, each a
            # VCF with the header): the reference's CPU path on the box's share
            # of host cores (SURVEY §8 d)
            P = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1, 16))
            cut = [0]
            for q in range(1, P):
                c = body.find(b"\n", max(len(body) * q // P, cut[-1])) + 1
                cut.append(c if c > 0 else len(body))
            cut.append(len(body))
            paths = []
            for q in range(P):
                pq = os.path.join(d, "p%d.vcf" % q)
                with open(pq, "wb") as f:
                    f.write(header + body[cut[q]:cut[q + 1]])
                paths.append(pq)
            t0 = time.perf_counter()
            procs = [subprocess.Popen([ref, "compress", pq, pq + "c"], stdout=subprocess.DEVNULL,
                                      stderr=subprocess.DEVNULL) for pq in paths]
            rcs = [pr.wait() for pr in procs]
            dtp = time.perf_counter() - t0
            same = all(r == 0 for r in rcs) and b"".join(open(pq + "c", "rb").read()[len(header):]
                                                         for pq in paths) == out
            par = {"value": round(gt / dtp / 1e9, 4), "unit": "GB/s", "cores": P, "kind": "reference",
                   "sample": "the same %d rows as %d byte-balanced shards, %d concurrent `main compress` "
                             "processes, wall time %.2f s" % (k, P, P, dtp), "output_identical": same}
    res = {"value": round(gt / dt / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": kind,
           "sample": "first %d rows of the rank-0 shard (%d GT bytes, %.1f MB file), `main compress` wall time %.2f s"
                     % (k, gt, (len(header) + len(body)) / 1e6, dt)}
    if par:
        res["parallel"] = par
    return (res, out, k)


def load_pmc(workload_key, name="pmc_k_encode.json"):
    """HBM bytes per launch from a committed rocprofv3 PMC summary
    (profiles/<name>, or profiles/<stem>_*.json for other workloads) when it
    was measured on this workload, else None."""
    import glob
    stem = os.path.splitext(name)[0]
    for p in [os.path.join(REPO, "profiles", name)] + sorted(glob.glob(os.path.join(REPO, "profiles", stem + "_*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") == workload_key:
            return d.get("hbm_bytes_per_launch")
    return None


def load_pmc_step(workload_key):
    """HBM bytes of the whole encode step (k_encode kernels + k_compact_out)
    per call, from the same committed PMC summary as load_pmc, or None."""
    import glob
    for p in [os.path.join(REPO, "profiles", "pmc_k_encode.json")] + sorted(
            glob.glob(os.path.join(REPO, "profiles", "pmc_k_encode_*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") == workload_key and "kernels" in d:
            return sum(v.get("hbm_bytes", 0) for v in d["kernels"].values())
    return None


def sample_header(S):
    return ("##fileformat=VCFv4.2\n##source=vcfc-mi355x bench\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT"
            + "".join("\tS%d" % i for i in range(S)) + "\n").encode()


def encoded_shard(args, torch, vcfc, workload, dev):
    """The synthetic batch and its records, both resident in HBM (GPU encoder)."""
    n, S = args.rows, args.samples
    rows = workload.DeviceRows(torch, vcfc, n, S, args.law, seed=1000, device=dev)
    ws_bytes = vcfc.workspace_size(n, rows.line_bytes)
    cap = vcfc.encode_bound(n, rows.line_bytes)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    recs = torch.empty(cap, dtype=torch.uint8, device=dev)
    rec = torch.empty(n + 1, dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    vcfc.encode_rows_device(rows.buf.data_ptr(), rows.line_off.data_ptr(), rows.line_len.data_ptr(), n,
                            rows.line_bytes, recs.data_ptr(), cap, rec.data_ptr(), ws.data_ptr(), ws_bytes,
                            err.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    del ws
    return rows, recs, rec, int(rec[n].item())


def cpu_reference_run(rows, recs, rec, args, verb_args):
    """Time the reference CLI (oracle/_ref/main; else the C restatement) on
    a .vcfc of the first --cpu-rows rows of the batch.  verb_args(path) ->
    argv tail, e.g. ["decompress", path, out].  Returns (seconds, rows, kind)."""
    k = min(args.cpu_rows, rows.n)
    body = recs[:int(rec[k].item())].cpu().numpy().tobytes()
    data = sample_header(rows.samples) + body
    ref = os.path.join(REPO, "oracle", "_ref", "main")
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        path = os.path.join(d, "s.vcfc")
        with open(path, "wb") as f:
            f.write(data)
        argv = verb_args(path)
        if os.path.exists(ref):
            with open(os.path.join(d, "stdout"), "wb") as so:
                t0 = time.perf_counter()
                r = subprocess.run([ref] + argv, stdout=so, stderr=subprocess.PIPE)
                dt = time.perf_counter() - t0
            if r.returncode != 0:
                raise RuntimeError("reference %s failed: %s" % (argv[0], r.stderr[-400:]))
            return dt, k, "reference"
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import golden_io as G
        t0 = time.perf_counter()
        if argv[0] == "decompress":
            st, _ = G.oracle_decompress(data, cap=len(data) * 8 + (1 << 20))
        else:
            st, _ = G.oracle_query(data, argv[2].encode(), cap=len(data) * 8 + (1 << 20))
        dt = time.perf_counter() - t0
        assert st == 0
        return dt, k, "port"


def measured_copy_gbs(torch, dev, nbytes=4 << 30):
    """Device-to-device copy rate on this GPU (read + write bytes / time):
    the practical HBM ceiling beside the 8 TB/s spec peak."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize(dev)
    gbs = 2 * nbytes * 5 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return round(gbs, 1)


def timed(torch, dev, args, step):
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
    return time.perf_counter() - t0, e0.elapsed_time(e1) / args.steps


def bench_decode(args, torch, vcfc, workload):
    """Row f1: decode the same synthetic batch (device-resident records made
    by the GPU encoder) back to VCF lines; every output byte is checked
    against the original rows on the GPU.  One GPU (replicas only)."""
    import numpy as np
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n, S = args.rows, args.samples
    rows, recs, rec, rec_bytes = encoded_shard(args, torch, vcfc, workload, dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    err = torch.empty(1, dtype=torch.int64, device=dev)
    dws_bytes = vcfc.decode_workspace_size(n)
    dws = torch.empty(dws_bytes, dtype=torch.uint8, device=dev)
    out_cap = rows.total_bytes + 64
    out = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    loff = torch.empty(n + 1, dtype=torch.int64, device=dev)

    def step():
        vcfc.decode_records_device(recs.data_ptr(), rec_bytes, rec.data_ptr(), n, S, out.data_ptr(), out_cap,
                                   loff.data_ptr(), dws.data_ptr(), dws_bytes, err.data_ptr(), stream)

    elapsed, ev_ms = timed(torch, dev, args, step)
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
           "config": {"workload": "%s %d samples x %d variants" % (law_name(args.law), S, n),
                      "record_bytes": rec_bytes, "line_bytes": total},
           "roofline": {"kernel": "k_dec_plan + k_dec_write", "bound": "hbm",
                        "achieved": round(alg / (ev_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / (ev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": load_pmc("%s/%dx%d" % (law_name(args.law), S, n), "pmc_k_dec.json"),
                        "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(ev_ms, 4)},
           "output_identical_to_input_rows": identical}
    if not args.no_cpu_baseline:
        dt, k, kind = cpu_reference_run(rows, recs, rec, args, lambda p: ["decompress", p, p + ".vcf"])
        res["cpu_baseline"] = {"value": round(4 * S * k / dt / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": kind,
                               "sample": "`main decompress` of the first %d records (%d GT bytes), wall time %.2f s"
                                         % (k, 4 * S * k, dt)}
    print(json.dumps(res), flush=True)


def bench_query(args, torch, vcfc, workload):
    """Row f2: range query over the same device-resident .vcfc records: match
    every record's CHROM/POS (k_query_match), then decode the selected ones
    (k_dec_plan + k_dec_write with the match flags).  The query selects
    --query-frac of the rows (a POS window in the middle of the batch); the
    output is checked byte-exact against those rows on the GPU."""
    import numpy as np
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n, S = args.rows, args.samples
    rows, recs, rec, rec_bytes = encoded_shard(args, torch, vcfc, workload, dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    a = int(n * (0.5 - args.query_frac / 2))
    b = min(n - 1, a + max(1, int(n * args.query_frac)) - 1)
    qs, qe = int(rows.pos[a]), int(rows.pos[b])
    ref = rows.chrom.encode()
    d_ref = torch.tensor(list(ref), dtype=torch.uint8, device=dev)
    flag = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    merr = torch.empty(1, dtype=torch.int64, device=dev)
    derr = torch.empty(1, dtype=torch.int64, device=dev)
    dws_bytes = vcfc.decode_workspace_size(n)
    dws = torch.empty(dws_bytes, dtype=torch.uint8, device=dev)
    lo = rows.line_off.cpu().numpy()
    sel_lines = int(lo[b + 1] if b + 1 < n else rows.total_bytes) - int(lo[a])
    out_cap = sel_lines + 64
    out = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    loff = torch.empty(n + 1, dtype=torch.int64, device=dev)

    def step():
        st = vcfc.query_match_device(recs.data_ptr(), rec.data_ptr(), n, d_ref.data_ptr(), len(ref), True, qs, qe,
                                     flag.data_ptr(), merr.data_ptr(), stream)
        vcfc.raise_for(st)
        vcfc.decode_selected_device(recs.data_ptr(), rec_bytes, rec.data_ptr(), flag.data_ptr(), n, S, out.data_ptr(),
                                    out_cap, loff.data_ptr(), dws.data_ptr(), dws_bytes, derr.data_ptr(), stream)

    elapsed, ev_ms = timed(torch, dev, args, step)
    e1 = int(merr.cpu().numpy().view(np.uint64)[0])
    e2 = int(derr.cpu().numpy().view(np.uint64)[0])
    total = int(loff[n].item())
    want = rows.buf[int(lo[a]):int(lo[a]) + sel_lines]
    identical = (e1 == vcfc.NO_ERROR and e2 == vcfc.NO_ERROR and total == sel_lines
                 and int(flag[:n].sum().item()) == b - a + 1 and bool(torch.equal(out[:total], want)))
    sel_rec = int(rec[b + 1].item()) - int(rec[a].item())
    # algorithmic bytes: per record its offset (8), LEN/REQ + CHROM\tPOS\t (read), its flag (write); the
    # selected records once more in full, their lines written, plus the line offsets
    fields = 8 + len(ref) + 1 + float(np.mean([len(str(p)) for p in rows.pos[:1000]])) + 1
    alg = int(n * (8 + fields + 1 + 8) + sel_rec + sel_lines)
    q = "%s:%d-%d" % (rows.chrom, qs, qe)
    res = {"metric": "queried .vcfc bytes/sec, range query over a 2504-sample x 1M-variant .vcfc (row f2)",
           "value": round(rec_bytes * args.steps / elapsed / 1e9, 2), "unit": "GB/s", "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
           "higher_is_better": True, "scaling": "replicas", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (generated and encoded in HBM)",
           "config": {"workload": "%s %d samples x %d variants, query %s (%d rows, %.1f%%)"
                                  % (law_name(args.law), S, n, q, b - a + 1,
                                     100.0 * (b - a + 1) / n),
                      "record_bytes": rec_bytes, "selected_record_bytes": sel_rec, "line_bytes": total},
           "roofline": {"kernel": "k_query_match + k_dec_plan + k_dec_write", "bound": "hbm",
                        "achieved": round(alg / (ev_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / (ev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": load_pmc("%s/%dx%d/%s" % (law_name(args.law), S, n, args.query_frac),
                                            "pmc_k_query.json"),
                        "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(ev_ms, 4)},
           "output_identical_to_selected_rows": identical}
    if not args.no_cpu_baseline:
        k = min(args.cpu_rows, n)
        ka = int(k * (0.5 - args.query_frac / 2))
        kb = min(k - 1, ka + max(1, int(k * args.query_frac)) - 1)
        kq = "%s:%d-%d" % (rows.chrom, int(rows.pos[ka]), int(rows.pos[kb]))
        dt, k, kind = cpu_reference_run(rows, recs, rec, args, lambda p: ["query", p, kq])
        kbytes = int(rec[k].item())
        res["cpu_baseline"] = {"value": round(kbytes / dt / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": kind,
                               "sample": "`main query %s` over the first %d records (%d .vcfc bytes), wall time %.2f s"
                                         % (kq, k, kbytes, dt)}
    print(json.dumps(res), flush=True)


def bench_ingest(args, torch, vcfc, workload):
    """Row f4: end-to-end `compress` of a VCF file on disk to a .vcfc file
    (vcfc_compress_file: reader threads -> pinned H2D -> GPU line index +
    encode -> writer thread).  The file holds --ingest-rows synthetic rows
    (written from HBM, so it sits in the page cache, as in a pipeline that
    has just produced it); the output is checked byte-for-byte against the
    GPU encoder's device-resident records."""
    import numpy as np
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    args.rows = args.ingest_rows
    n, S = args.rows, args.samples
    rows, recs, rec, rec_bytes = encoded_shard(args, torch, vcfc, workload, dev)
    header = sample_header(S)
    want = header + recs[:rec_bytes].cpu().numpy().tobytes()
    del recs
    tmp = tempfile.mkdtemp(dir="/tmp")
    src, dst = os.path.join(tmp, "in.vcf"), os.path.join(tmp, "out.vcfc")
    try:
        with open(src, "wb") as f:
            f.write(header)
            step = 1 << 28
            for a in range(0, rows.total_bytes, step):
                f.write(rows.buf[a:min(rows.total_bytes, a + step)].cpu().numpy().tobytes())
        in_bytes = len(header) + rows.total_bytes
        # pinned H2D peak of this box (the bound of the pipeline's transfer stage)
        hb = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
        db = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
        db.copy_(hb, non_blocking=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(5):
            db.copy_(hb, non_blocking=True)
        torch.cuda.synchronize(dev)
        h2d = 5 * (256 << 20) / (time.perf_counter() - t0) / 1e9
        del hb, db
        ctx = vcfc.Context(0)
        for _ in range(args.warmup):
            ctx.compress_file(src, dst)
        elapsed = 0.0
        for _ in range(args.steps):   # each step writes a fresh output file (the old one is removed untimed)
            os.unlink(dst)
            t0 = time.perf_counter()
            ctx.compress_file(src, dst)
            elapsed += time.perf_counter() - t0
        identical = open(dst, "rb").read() == want
        ctx.close()
        res = {"metric": "end-to-end input GT bytes/sec, VCF file -> .vcfc file (compress(), BASELINE configs[2]; row f4)",
               "value": round(rows.gt_bytes * args.steps / elapsed / 1e9, 3), "unit": "GB/s", "n_gpus": 1,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
               "higher_is_better": True, "scaling": "replicas", "vs_baseline": None, "dtype": "u8",
               "data": "synthetic (generated in HBM, written to a file in the page cache)",
               "config": {"workload": "%s %d samples x %d variants, %.2f GB file"
                                      % (law_name(args.law), S, n, in_bytes / 1e9),
                          "input_bytes": in_bytes, "output_bytes": len(want)},
               "roofline": {"kernel": "pipeline (file read + H2D + index + encode + D2H + write)", "bound": "pcie",
                            "achieved": round(in_bytes * args.steps / elapsed / 1e9, 2), "peak": round(h2d, 1),
                            "unit": "GB/s", "frac": round(in_bytes * args.steps / elapsed / 1e9 / h2d, 4),
                            "traffic": None, "peak_note": "pinned H2D of this box, measured"},
               "output_identical_to_gpu_records": identical}
        if not args.no_cpu_baseline:
            k = min(args.cpu_rows, n)
            end = int(rows.line_off[k].item()) if k < n else rows.total_bytes
            with open(os.path.join(tmp, "s.vcf"), "wb") as f:
                f.write(header)
                f.write(rows.buf[:end].cpu().numpy().tobytes())
            ref = os.path.join(REPO, "oracle", "_ref", "main")
            if os.path.exists(ref):
                t0 = time.perf_counter()
                r = subprocess.run([ref, "compress", os.path.join(tmp, "s.vcf"), os.path.join(tmp, "s.vcfc")],
                                   capture_output=True)
                dt = time.perf_counter() - t0
                if r.returncode == 0:
                    res["cpu_baseline"] = {"value": round(4 * S * k / dt / 1e9, 4), "unit": "GB/s", "cores": 1,
                                           "kind": "reference",
                                           "sample": "`main compress` of the first %d rows (file -> file), %.2f s"
                                                     % (k, dt)}
        print(json.dumps(res), flush=True)
    finally:
        for f in os.listdir(tmp):
            os.unlink(os.path.join(tmp, f))
        os.rmdir(tmp)


def bench_devfile(args, torch, vcfc, workload):
    """compress() of the configs[1] file with its bytes already in HBM
    (vcfc_compress_device): the GPU line index ('\n' scan, data / '#' line
    tables) and the encoder over the whole file, in chunks of whole lines, the
    .vcfc bytes left in HBM -- "device-resident file bytes -> records", the
    headline step plus finding the lines.  The output is checked byte for byte
    on the GPU against header + the encoder's records of the same rows."""
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n, S = args.rows, args.samples
    rows, recs, rec, rec_bytes = encoded_shard(args, torch, vcfc, workload, dev)
    header = sample_header(S)
    H = len(header)
    N = H + rows.total_bytes
    d_file = torch.empty(N, dtype=torch.uint8, device=dev)
    d_file[:H] = torch.frombuffer(bytearray(header), dtype=torch.uint8).to(dev)
    d_file[H:] = rows.buf[:rows.total_bytes]
    want_len = H + rec_bytes
    cap = int(vcfc.lib().vcfc_compress_bound(N))
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)   # the call runs on the context's own stream
    ctx = vcfc.Context(0)
    if args.dev_chunk:
        ctx.set_ingest_chunk(args.dev_chunk)
    ctx.set_line_index(args.line_index)
    ctx.set_deferred_records(args.deferred_records == "on")
    for _ in range(args.warmup):
        st, k, _ = ctx.compress_device(d_file.data_ptr(), N, d_out.data_ptr(), cap)
        assert st == 0 and k == want_len, (st, k, want_len)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.compress_device(d_file.data_ptr(), N, d_out.data_ptr(), cap)
    elapsed = time.perf_counter() - t0   # (the call is synchronous)
    identical = bool(torch.equal(d_out[:H], d_file[:H])) and bool(torch.equal(d_out[H:want_len], recs[:rec_bytes]))
    ctx.close()
    ms = elapsed * 1e3 / args.steps
    hop = args.line_index == "hop"
    alg = N + want_len   # the file read once, the output written once
    res = {"metric": "input GT bytes/sec, device-resident VCF file bytes -> .vcfc bytes (line index + encode)",
           "value": round(rows.gt_bytes / (ms * 1e-3) / 1e9, 2), "unit": "GB/s", "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
           "scaling": "replicas", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (generated in HBM; header + data lines as one device buffer)",
           "config": {"workload": "%s %d samples x %d variants, %.2f GB file in HBM (BASELINE configs[1])"
                                  % (law_name(args.law), S, n, N / 1e9),
                      "file_bytes": N, "output_bytes": want_len,
                      "deferred_records": args.deferred_records == "on",
                      "chunk": ("%d bytes of whole lines per line index + encode" % args.dev_chunk) if args.dev_chunk
                               else "the whole file (one line index, one encode)",
                      "line_index": ("hop (line ends guessed from the header's sample count and the lines' "
                                     "mean length, ~0.3 KiB read per chr22-shaped line, checked by the encoder)") if hop else "scan of every byte (--line-index scan)"},
           "roofline": {"kernel": "line index + encoder (whole step)", "bound": "hbm",
                        "achieved": round(alg / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": load_pmc("%s/%dx%d/%s%s" % (law_name(args.law), S, n, args.line_index,
                                                                  "" if args.deferred_records == "on" else "/nodefer"),
                                            "pmc_devfile.json"),
                        "algorithmic_bytes_per_step": alg,
                        "note": "file bytes read once + output written once (the scan index reads the file "
                                "a second time)"},
           "output_identical_to_header_plus_records": identical}
    print(json.dumps(res), flush=True)


def bench_sparse(args, torch, vcfc, workload):
    """Rows a7-a9 + f3: `sparsify` of a .vcfc file (GPU plan + one pwritev
    per record) and `sparse-query` of the middle --query-frac of its rows
    (host walk of the dist_to_next hops, GPU decode of the walked records)
    over --sparse-rows GPU-encoded rows.  Both are file -> file paths bound by
    host I/O (one pread / pwrite per record), so there is no kernel roofline;
    the reference CLI runs beside them on the same files."""
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    args.rows = args.sparse_rows
    n, S = args.rows, args.samples
    rows, recs, rec, rec_bytes = encoded_shard(args, torch, vcfc, workload, dev)
    header = sample_header(S)
    tmp = tempfile.mkdtemp(dir="/tmp")
    src, sp = os.path.join(tmp, "in.vcfc"), os.path.join(tmp, "out.sparse")
    with open(src, "wb") as f:
        f.write(header)
        f.write(recs[:rec_bytes].cpu().numpy().tobytes())
    del recs
    a = int(n * (0.5 - args.query_frac / 2))
    b = min(n - 1, a + max(1, int(n * args.query_frac)) - 1)
    q = "%s:%d-%d" % (rows.chrom, int(rows.pos[a]), int(rows.pos[b]))
    lo = rows.line_off.cpu().numpy()
    want = rows.buf[int(lo[a]):int(lo[b + 1]) if b + 1 < n else rows.total_bytes].cpu().numpy().tobytes()
    ref = os.path.join(REPO, "oracle", "_ref", "main")
    try:
        with vcfc.Context(0) as ctx:
            ts = []
            for k in range(max(1, args.warmup) + 3):
                if os.path.exists(sp):
                    os.unlink(sp)
                t0 = time.perf_counter()
                ctx.sparsify_file(src, sp)
                ts.append(time.perf_counter() - t0)
            t_sp = min(ts[max(1, args.warmup):])
            qp = os.path.join(tmp, "q.out")
            for _ in range(args.warmup):
                st, got = ctx.sparse_query_status(sp, q)
            identical = st == 0 and got == want
            # a fresh output file per step (as `main sparse-query ... > file`); removed after timing
            fds = [os.open("%s.%d" % (qp, k), os.O_CREAT | os.O_TRUNC | os.O_WRONLY, 0o600) for k in range(args.steps)]
            t0 = time.perf_counter()
            for fd in fds:
                ctx.sparse_query_file(sp, q, fd)
            elapsed = time.perf_counter() - t0
            for fd in fds:
                os.close(fd)
        res = {"metric": "sparse-query output VCF bytes/sec over a sparsified 2504-sample .vcfc (rows a7-a9, f3)",
               "value": round(len(want) * args.steps / elapsed / 1e9, 3), "unit": "GB/s", "n_gpus": 1,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
               "higher_is_better": True, "scaling": "replicas", "vs_baseline": None, "dtype": "u8",
               "data": "synthetic (generated and encoded in HBM, files in the page cache)",
               "config": {"workload": "chr22-shaped %d samples x %d variants, sparse-query %s (%d records)"
                                      % (S, n, q, b - a + 1),
                          "vcfc_bytes": len(header) + rec_bytes, "query_output_bytes": len(want)},
               "records_per_sec": round((b - a + 1) * args.steps / elapsed, 1),
               "sparsify": {"seconds": round(t_sp, 4), "records_per_sec": round(n / t_sp, 1),
                            "vcfc_bytes_per_sec": round((len(header) + rec_bytes) / t_sp / 1e9, 4)},
               "roofline": None, "roofline_note": "host-I/O bound: one pread (query) / pwritev (sparsify) per record",
               "output_identical_to_selected_rows": identical}
        if not args.no_cpu_baseline and os.path.exists(ref):
            with open(os.path.join(tmp, "r.out"), "wb") as so:
                t0 = time.perf_counter()
                r = subprocess.run([ref, "sparse-query", sp, q], stdout=so, stderr=subprocess.PIPE)
                dt = time.perf_counter() - t0
            same = r.returncode == 0 and open(os.path.join(tmp, "r.out"), "rb").read() == want
            k = min(n, 3000)
            ksrc, ksp = os.path.join(tmp, "k.vcfc"), os.path.join(tmp, "k.sparse")
            with open(src, "rb") as f:
                kb = f.read(len(header) + int(rec[k].item()))
            with open(ksrc, "wb") as f:
                f.write(kb)
            t0 = time.perf_counter()
            r2 = subprocess.run([ref, "sparsify", ksrc, ksp], capture_output=True)
            dt2 = time.perf_counter() - t0
            res["cpu_baseline"] = {"value": round(len(want) / dt / 1e9, 4), "unit": "GB/s", "cores": 1,
                                   "kind": "reference",
                                   "sample": "`main sparse-query %s` on the same sparse file, wall time %.3f s" % (q, dt),
                                   "output_identical": same,
                                   "sparsify": {"records": k, "seconds": round(dt2, 3),
                                                "records_per_sec": round(k / dt2, 1), "rc": r2.returncode}}
        print(json.dumps(res), flush=True)
    finally:
        for f in os.listdir(tmp):
            os.unlink(os.path.join(tmp, f))
        os.rmdir(tmp)


def bench_biobank_shard(args):
    """configs[3] as a whole shard: rank r of N encodes rows [R*r/N, R*(r+1)/N)
    of the R = --rows-total row dataset (100k samples) as back-to-back
    batches of --rows rows.  Every batch is generated in HBM (same prefixes,
    a new genotype seed per batch; generation is outside the timed encode),
    encoded, its records digested on the GPU (vcfc_record_hash_device) and
    folded into a shard checksum; two rows per batch are re-encoded by the
    CPU checker (oracle) and compared byte for byte, and each pass checks
    EVERY record of one whole batch (a different batch per pass: pass p
    takes batch 7p mod nb) and --sample-rows random rows of every other
    batch against the checker's threaded digests and sizes (SURVEY §7 hard
    part 7: per-row hashes plus a sampled CPU re-encode across the shard).
    One step = the whole shard; `ms_per_step` and `value` use the summed
    encode time of its batches (HIP events on the encode stream), max over
    ranks; the wall time including generation and checks is reported too."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import vcfc
    import workload
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rehearsal = os.environ.get("VCFC_BENCH_REHEARSAL") == "1"
    check_world(args, torch, world, local, rehearsal)
    dev = torch.device("cuda:%d" % (0 if rehearsal else local))
    torch.cuda.set_device(dev)
    cdev = torch.device("cpu") if rehearsal else dev
    if world > 1:
        init_dist(dist, rehearsal, dev)
    rccl = rccl_report(torch, dist, dev, cdev, world, rehearsal)
    R, B, S = args.rows_total, args.rows, args.samples
    lo, hi = R * rank // world, R * (rank + 1) // world
    nb = (hi - lo + B - 1) // B
    import dist_compress as D
    rows = D.setup_all_or_none(rank, lambda v: gather_ints(torch, dist, cdev, world, v),
                               lambda: workload.DeviceRows(torch, vcfc, B, S, args.law, seed=5000, device=dev, row0=lo))
    ll = rows.line_len_host.astype(np.int64)
    lb_prefix = np.concatenate([[0], np.cumsum(ll)])          # line bytes of the first k rows
    gt_prefix = np.concatenate([[0], np.cumsum(rows.gt_row)])  # GT bytes of the first k rows
    ws_bytes = vcfc.workspace_size(B, rows.line_bytes)
    cap = vcfc.encode_bound(B, rows.line_bytes)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    rec = torch.empty(B + 1, dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    dig = torch.empty(B, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import golden_io as G   # the CPU checker (oracle), verification only
    rng = np.random.default_rng(rank)
    line_off_host = rows.line_off.cpu().numpy()
    cpu_threads = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    verified_batches = []
    sampled_batches = set()

    def verify_batch(b, n, d):
        """every record of batch b: the oracle's size and digest (threaded)"""
        buf = rows.buf[:rows.total_bytes].cpu().numpy()
        st, size, want = G.oracle_encode_rows_hash(buf, line_off_host[:n], rows.line_len_host[:n], threads=cpu_threads)
        del buf
        r = rec[:n + 1].cpu().numpy().astype(np.uint64)
        bad = np.nonzero((st != 0) | (size.astype(np.uint64) != np.diff(r)) | (want != d))[0]
        if bad.size:
            raise RuntimeError("batch %d: rows %s differ from the CPU checker" % (b, bad[:8].tolist()))
        verified_batches.append(b)
        return n

    def verify_sample(b, n, d, k):
        """k random rows of batch b (gathered on the GPU, ~k x 400 KB to the
        host): the oracle's sizes and digests of its own encode against the
        GPU's in-place digests d."""
        idx = np.sort(rng.choice(n, size=min(k, n), replace=False))
        offs = line_off_host[idx].astype(np.int64)
        lens = rows.line_len_host[idx].astype(np.int64)
        blob = torch.cat([rows.buf[int(o):int(o) + int(ln)] for o, ln in zip(offs, lens)]).cpu().numpy()
        loc = np.concatenate([[0], np.cumsum(lens)[:-1]])
        st, size, want = G.oracle_encode_rows_hash(blob, loc, lens, threads=cpu_threads)
        r = rec[:n + 1].cpu().numpy().astype(np.uint64)
        bad = np.nonzero((st != 0) | (size.astype(np.uint64) != (r[idx + 1] - r[idx])) | (want != d[idx]))[0]
        if bad.size:
            raise RuntimeError("batch %d: rows %s differ from the CPU checker" % (b, idx[bad[:8]].tolist()))
        sampled_batches.add(b)
        return len(idx)

    def shard_pass(check, p=0):
        enc_ms, gt, recb, checked = 0.0, 0, 0, 0
        csum, cxor = 0, 0
        for b in range(nb):
            n = min(B, hi - lo - b * B)
            rows.resynth(seed=7000 + (lo // B) + b)       # the batch's genotypes (input production, untimed)
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            vcfc.encode_rows_device(rows.buf.data_ptr(), rows.line_off.data_ptr(), rows.line_len.data_ptr(), n,
                                    int(lb_prefix[n]), out.data_ptr(), cap, rec.data_ptr(), ws.data_ptr(), ws_bytes,
                                    err.data_ptr(), stream)
            e1.record()
            torch.cuda.synchronize(dev)
            enc_ms += e0.elapsed_time(e1)
            e = int(err.cpu().numpy().view(np.uint64)[0])
            if e != vcfc.NO_ERROR:
                raise RuntimeError("batch %d: row error %x" % (b, e))
            gt += int(gt_prefix[n])
            recb += int(rec[n].item())
            if not check:
                continue
            vcfc.record_hash_device(out.data_ptr(), rec.data_ptr(), n, dig.data_ptr(), stream)
            d = dig[:n].cpu().numpy().view(np.uint64)
            csum = (csum + int(d.sum(dtype=np.uint64))) & ((1 << 64) - 1)
            cxor ^= int(np.bitwise_xor.reduce(d))
            if b == (7 * p) % nb:
                full_rows[0] += verify_batch(b, n, d)
            elif args.sample_rows:
                full_rows[0] += verify_sample(b, n, d, args.sample_rows)
            for i in rng.integers(0, n, 2):
                line = rows.host_lines([int(i)])[0]
                got = out[int(rec[i].item()):int(rec[i + 1].item())].cpu().numpy().tobytes()
                st, want = G.oracle_encode_line(line)
                if st != 0 or got != want or G.oracle_hash64(want) != int(d[i]):
                    raise RuntimeError("batch %d row %d differs from the CPU checker" % (b, int(i)))
                checked += 1
        return enc_ms, gt, recb, checked, (csum, cxor)

    for _ in range(args.warmup):
        shard_pass(False)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    enc_ms, gt, recb, checked, ck = 0.0, 0, 0, 0, None
    full_rows = [0]
    for p in range(args.steps):
        m, gt, recb, c, k = shard_pass(True, p)
        enc_ms += m
        checked += c
        if ck is not None and k != ck:
            raise RuntimeError("shard checksum changed between passes")
        ck = k
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    t = torch.tensor([enc_ms / args.steps, wall / args.steps], dtype=torch.float64, device=cdev)
    g = torch.tensor([gt], dtype=torch.int64, device=cdev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(g)
    ms, wall_s = float(t[0].item()), float(t[1].item())
    gt_all = int(g.item())
    res = {"metric": "input GT bytes/sec encoded, 100k-sample x 5M-variant VCF, row-sharded",
           "value": round(gt_all / (ms * 1e-3) / 1e9, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "u8", "data": "synthetic (generated in HBM, batch by batch)",
           "config": {"workload": "%s %d samples x %d variants, whole shard per GPU: %d-row batches back to back "
                                  "(BASELINE configs[3])" % (law_name(args.law), S, R, B),
                      "rows_total": R, "rows_per_gpu": hi - lo, "batches_per_gpu": nb, "gt_bytes_total": gt_all,
                      "record_bytes_rank0": recb, "parallelism": "row shards x%d" % world},
           "timing": "ms_per_step = summed HIP-event encode time of the shard's batches (generation and checks "
                     "excluded), max over ranks; wall_s_per_step includes them",
           "wall_s_per_step": round(wall_s, 3),
           "verification": {"records_digested_per_pass": hi - lo,
                            "rows_verified": full_rows[0] + checked,
                            "rows_verified_by_oracle_digest": full_rows[0],
                            "batches_verified_every_record": verified_batches,
                            "batches_verified_by_sample": len(sampled_batches),
                            "sample_rows_per_batch": args.sample_rows,
                            "rows_reencoded_byte_for_byte": checked,
                            "shard_checksum_rank0": "%016x:%016x (determinism across passes, not parity)" % ck},
           "rccl_world": rccl}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_distfile(args):
    """Row (e) end to end: the sharded `compress` of one VCF file into one
    .vcfc file, as vcf-compression_amd/dist_compress.py runs it (one process
    per GPU).  Every rank contributes --ingest-rows chr22-shaped rows (weak
    scaling) to one input file (written untimed, so it sits in the page
    cache); a step is the whole job: every rank streams its line-aligned
    byte range through the ingest pipeline (reader threads, pinned H2D, GPU
    line index + encode, D2H), rank 0 writes in place, the other ranks hold
    their output in host memory, one all-gather of the byte counts gives the
    offsets, the held bytes are written there once; a fresh output file per
    step.  Time = max over ranks of the wall time between barriers.  After
    timing, every rank checks its rows' slice of the output file against its
    own GPU-encoded records (and rank 0 the header)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import vcfc
    import workload
    import dist_compress as D
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rehearsal = os.environ.get("VCFC_BENCH_REHEARSAL") == "1"
    check_world(args, torch, world, local, rehearsal)
    dev = torch.device("cuda:%d" % (0 if rehearsal else local))
    torch.cuda.set_device(dev)
    cdev = torch.device("cpu") if rehearsal else dev
    if world > 1:
        init_dist(dist, rehearsal, dev)
    rccl = rccl_report(torch, dist, dev, cdev, world, rehearsal)

    def allgather(vals):
        if world == 1:
            return [list(vals)]
        t = torch.tensor(vals, dtype=torch.int64, device=cdev)
        o = torch.empty(world * len(vals), dtype=torch.int64, device=cdev)
        dist.all_gather_into_tensor(o, t)
        return o.view(world, len(vals)).cpu().tolist()

    def barrier():
        if world > 1:
            dist.barrier()

    n, S = args.ingest_rows, args.samples
    rows = D.setup_all_or_none(rank, allgather, lambda: workload.DeviceRows(torch, vcfc, n, S, args.law,
                                                                            seed=2000 + rank, device=dev,
                                                                            row0=rank * n))
    ws_bytes = vcfc.workspace_size(n, rows.line_bytes)
    cap = vcfc.encode_bound(n, rows.line_bytes)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    recs = torch.empty(cap, dtype=torch.uint8, device=dev)
    rec = torch.empty(n + 1, dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    vcfc.encode_rows_device(rows.buf.data_ptr(), rows.line_off.data_ptr(), rows.line_len.data_ptr(), n,
                            rows.line_bytes, recs.data_ptr(), cap, rec.data_ptr(), ws.data_ptr(), ws_bytes,
                            err.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    assert int(err.cpu().numpy().view(np.uint64)[0]) == vcfc.NO_ERROR
    my_rec = recs[:int(rec[n].item())].cpu().numpy().tobytes()
    del ws, recs
    header = sample_header(S)
    g = allgather([rows.total_bytes, len(my_rec), rows.gt_bytes])
    in_off = len(header) + sum(x[0] for x in g[:rank])
    out_off = len(header) + sum(x[1] for x in g[:rank])
    gt_all = sum(x[2] for x in g)
    ip, op = os.path.join(args.dist_dir, "in.vcf"), os.path.join(args.dist_dir, "out.vcfc")
    if rank == 0:
        os.makedirs(args.dist_dir, exist_ok=True)
        with open(ip, "wb") as f:
            f.write(header)
    barrier()
    body = rows.buf[:rows.total_bytes].cpu().numpy()
    fd = os.open(ip, os.O_WRONLY)
    try:
        mv, o = memoryview(body), 0
        while o < len(body):
            o += os.pwrite(fd, mv[o:o + (1 << 30)], in_off + o)
    finally:
        os.close(fd)
    del body, rows
    torch.cuda.empty_cache()
    barrier()
    ctx = vcfc.Context(0 if rehearsal else local)
    hold = vcfc.hold_bytes()

    def hold_out(path, off, length):
        return ctx.compress_range_held(path, off, length, mem_bound=hold, spill_dir=args.dist_dir)

    def step():
        if rank == 0:
            if os.path.exists(op):
                os.unlink(op)
            open(op, "wb").close()
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        st, total, line = D.compress_shard(ip, op, rank, world, ctx.compress_range, hold_out, allgather)
        torch.cuda.synchronize(dev)
        barrier()
        dt = time.perf_counter() - t0
        if st:
            raise RuntimeError("sharded compress failed: status %d line %d" % (st, line))
        return dt, total

    for _ in range(args.warmup):
        step()
    tot_s = 0.0
    for _ in range(args.steps):
        dt, total = step()
        tot_s += dt
    t = torch.tensor([tot_s / args.steps], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    sec = float(t[0].item())
    # the output file: header (rank 0) + each rank's records at its offset
    with open(op, "rb") as f:
        ok = True
        if rank == 0:
            ok = f.read(len(header)) == header
        f.seek(out_off)
        ok = ok and f.read(len(my_rec)) == my_rec
        size_ok = os.path.getsize(op) == len(header) + sum(x[1] for x in g)
    okt = allgather([int(ok and size_ok)])
    ctx.close()
    res = {"metric": "input GT bytes/sec, sharded VCF file -> .vcfc file (row e end to end)",
           "value": round(gt_all / sec / 1e9, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(sec * 1e3, 2), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u8", "data": "synthetic (written from HBM; input file in the page cache)",
           "config": {"workload": "%s %d samples x %d variants per GPU, one file of %d rows"
                                  % (law_name(args.law), S, n, n * world),
                      "input_bytes": len(header) + sum(x[0] for x in g),
                      "output_bytes": len(header) + sum(x[1] for x in g),
                      "hold_bytes_per_rank_max": hold,
                      "parallelism": "byte-range shards x%d, all-gather of shard sizes%s"
                                     % (world, " (rehearsal: gloo, one GPU)" if rehearsal else "")},
           "timing": "wall time between barriers per step: read + H2D + line index + encode + D2H + write "
                     "(rank 0 in place, other ranks held then placed at the all-gathered offset), max over ranks",
           "output_identical_to_gpu_records": all(x[0] == 1 for x in okt),
           "rccl_world": rccl}
    if rank == 0:
        print(json.dumps(res), flush=True)
        if not res["output_identical_to_gpu_records"]:
            sys.exit(1)
    if world > 1:
        dist.destroy_process_group()


def strong_summary(per_rank, elapsed, steps, k_ms_rank0, rows_total, workload_name):
    """The `strong` object of a --gpus N > 1 encode line: the N=1 line's
    dataset (rows_total rows) split over the ranks.  per_rank: [rows, GT
    bytes, record bytes] of every rank; elapsed: max over ranks of the K
    timed steps (barrier + synchronize on both sides)."""
    rows = [int(r[0]) for r in per_rank]
    if sum(rows) != rows_total:
        raise RuntimeError("strong split lost rows: %s != %d" % (rows, rows_total))
    gt = sum(int(r[1]) for r in per_rank)
    return {"value": round(gt * steps / elapsed / 1e9, 2), "unit": "GB/s", "scaling": "strong",
            "ms_per_step": round(elapsed * 1e3 / steps, 4), "rows_total": rows_total, "rows_per_rank": rows,
            "gt_bytes_total": gt, "record_bytes_total": sum(int(r[2]) for r in per_rank),
            "k_encode_ms_rank0": round(k_ms_rank0, 4),
            "dataset": "%s, the N=1 line's %d-row batch (seed 1000) cut into contiguous row ranges, "
                       "byte-identical to it (workload.DeviceRows rows_of)" % (workload_name, rows_total)}


SHARDED_MODES = ("encode", "biobank", "distfile")


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_argv(n, argv, port):
    """The command that runs this bench as N ranks, one process per GPU:
    torch.distributed.run on this node, rendezvous on 127.0.0.1.  `argv` is
    bench.py's own argument list, passed through unchanged (each rank then
    sees WORLD_SIZE == --gpus)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
            "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + list(argv)


def launch_ranks(args, argv):
    """`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the
    environment: start the N ranks as a CHILD process (this parent has not
    imported torch or touched the GPU, and never execs), wait for it and
    return its exit code.  Rank 0's JSON line reaches our stdout directly."""
    if args.mode not in SHARDED_MODES:
        sys.stderr.write("bench.py: --mode %s runs on one GPU; --gpus %d applies to --mode %s\n"
                         % (args.mode, args.gpus, "/".join(SHARDED_MODES)))
        return 2
    cmd = launcher_argv(args.gpus, argv, free_port())
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def check_world(args, torch, world, local, rehearsal):
    """Inside a rank: the world is the --gpus the run asked for, and (outside
    the one-GPU rehearsal) every rank owns a distinct device."""
    if world != args.gpus:
        raise RuntimeError("WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    if world > 1 and not rehearsal:
        if torch.cuda.device_count() < world:
            raise RuntimeError("%d ranks but only %d visible GPUs" % (world, torch.cuda.device_count()))
        if not 0 <= local < torch.cuda.device_count():
            raise RuntimeError("LOCAL_RANK %d out of range" % local)


def init_dist(dist, rehearsal, dev):
    """One process group per run: RCCL on the rank's device (gloo with host
    tensors in the one-GPU rehearsal), every collective bounded by
    dist_compress.dist_timeout() (120 s), so a rank that dies ends the run
    with an error, not a wait past the driver's limit."""
    import dist_compress as D
    D.init_group(dist, "gloo" if rehearsal else "nccl", None if rehearsal else dev)


def gather_ints(torch, dist, cdev, world, vals):
    if world == 1:
        return [list(vals)]
    t = torch.tensor(vals, dtype=torch.int64, device=cdev)
    o = torch.empty(world * len(vals), dtype=torch.int64, device=cdev)
    dist.all_gather_into_tensor(o, t)
    return o.view(world, len(vals)).cpu().tolist()


def world_devices(torch, dist, dev, cdev, world):
    """PCI (domain, bus, device) of every rank's GPU, all-gathered: the run's
    proof that its N ranks sit on N distinct devices."""
    p = torch.cuda.get_device_properties(dev)
    me = [int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id)]
    if world == 1:
        return [me]
    t = torch.tensor(me, dtype=torch.int64, device=cdev)
    o = torch.empty(world * 3, dtype=torch.int64, device=cdev)
    dist.all_gather_into_tensor(o, t)
    return o.view(world, 3).cpu().tolist()


def rccl_report(torch, dist, dev, cdev, world, rehearsal):
    devs = world_devices(torch, dist, dev, cdev, world)
    distinct = len({tuple(d) for d in devs}) == world
    if world > 1 and not rehearsal and not distinct:
        raise RuntimeError("ranks share a GPU: %s" % devs)
    return {"world": world, "backend": ("gloo (one-GPU rehearsal)" if rehearsal else "nccl (RCCL)")
            if world > 1 else None,
            "devices_pci": ["%04x:%02x:%02x" % tuple(d) for d in devs], "distinct_devices": distinct}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, sys.argv[1:])
    if args.mode == "biobank" and args.rows_total:
        return bench_biobank_shard(args)
    if args.mode == "distfile":
        return bench_distfile(args)
    if args.mode not in ("encode", "biobank"):
        import torch
        import vcfc
        import workload
        fn = {"decode": bench_decode, "query": bench_query, "ingest": bench_ingest, "sparse": bench_sparse,
              "devfile": bench_devfile}[args.mode]
        return fn(args, torch, vcfc, workload)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch          # before libvcfc: one HIP runtime per process
    import torch.distributed as dist
    import vcfc
    import workload

    # VCFC_BENCH_REHEARSAL=1 rehearses the N > 1 path on one GPU: every rank on
    # cuda:0, gloo with host tensors for the collectives (RCCL refuses two
    # ranks on one device).  Never used for a reported number.
    rehearsal = os.environ.get("VCFC_BENCH_REHEARSAL") == "1"
    check_world(args, torch, world, local, rehearsal)
    dev = torch.device("cuda:%d" % (0 if rehearsal else local))
    torch.cuda.set_device(dev)
    cdev = torch.device("cpu") if rehearsal else dev   # collective tensors
    if world > 1:
        init_dist(dist, rehearsal, dev)
    rccl = rccl_report(torch, dist, dev, cdev, world, rehearsal)
    S = args.samples
    rows_asked = args.rows
    if rehearsal and args.mode == "encode" and args.scaling == "weak" and world > 4:
        # all ranks share the one GPU: 1M rows each (~43 GB of HBM per rank)
        # fit 4 ranks, so the weak phase of a wider rehearsal takes 4M rows
        # in all; the strong phase splits the full 1M-row dataset as asked
        args.rows = 4 * rows_asked // world
    import dist_compress as D

    def phase(n, make_rows):
        """Encode one n-row batch per rank: W untimed steps, then K steps
        bracketed by barrier + synchronize; returns the max-over-ranks
        wall time with the batch, its buffers and the stage timings."""
        def setup():
            rows = make_rows()
            ws_bytes = vcfc.workspace_size(n, rows.line_bytes)
            cap = vcfc.encode_bound(n, rows.line_bytes)
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
            out = torch.empty(cap, dtype=torch.uint8, device=dev)
            rec = torch.empty(n + 1, dtype=torch.int64, device=dev)
            err = torch.empty(1, dtype=torch.int64, device=dev)
            return rows, ws_bytes, cap, ws, out, rec, err
        # a rank whose setup fails (out of memory, no device) makes every rank
        # exit non-zero here, before the first all-gather of shard sizes
        rows, ws_bytes, cap, ws, out, rec, err = D.setup_all_or_none(
            rank, lambda v: gather_ints(torch, dist, cdev, world, v), setup)
        counts = torch.empty(world, dtype=torch.int64, device=cdev)
        timer = vcfc.StageTimer()
        stream = torch.cuda.current_stream(dev).cuda_stream

        def step(timed):
            f = timer.encode if timed else vcfc.encode_rows_device
            f(rows.buf.data_ptr(), rows.line_off.data_ptr(), rows.line_len.data_ptr(), n, rows.line_bytes,
              out.data_ptr(), cap, rec.data_ptr(), ws.data_ptr(), ws_bytes, err.data_ptr(), stream)
            if world > 1:
                # stitch: every rank learns every shard's record bytes -> its file offset
                dist.all_gather_into_tensor(counts, rec[n:n + 1].to(cdev))

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
        try:
            deferred = vcfc.encode_deferred_rows(ws.data_ptr(), n, rows.line_bytes, stream)
        except RuntimeError:   # (an A/B build of the library without the export)
            deferred = None
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        e = int(err.cpu().numpy().view(np.uint64)[0])
        if e != vcfc.NO_ERROR:
            raise RuntimeError("encode reported row error %x" % e)
        return dict(elapsed=elapsed, stages=stages, calls=calls, deferred=deferred, rows=rows, out=out, rec=rec)

    if args.scaling == "strong":
        # the --rows rows of the N=1 line's dataset split over the ranks: each
        # rank generates its contiguous slice of that one batch, byte for byte
        # (workload.DeviceRows rows_of; the total work is fixed)
        r0, r1 = args.rows * rank // world, args.rows * (rank + 1) // world
        n = r1 - r0
        P = phase(n, lambda: workload.DeviceRows(torch, vcfc, n, S, args.law, seed=1000, device=dev,
                                                 rows_of=(args.rows, r0)))
    else:
        r0, r1 = rank * args.rows, (rank + 1) * args.rows
        n = r1 - r0
        P = phase(n, lambda: workload.DeviceRows(torch, vcfc, n, S, args.law, seed=1000 + rank, device=dev,
                                                 row0=r0))
    elapsed, stages, calls, deferred = P["elapsed"], P["stages"], P["calls"], P["deferred"]
    rows, out, rec = P["rows"], P["out"], P["rec"]

    copy_gbs = measured_copy_gbs(torch, dev)
    out_bytes = int(rec[n].item())
    ms_step = elapsed * 1e3 / args.steps
    gt = torch.tensor([rows.gt_bytes], dtype=torch.int64, device=cdev)
    if world > 1:
        dist.all_reduce(gt)   # GT bytes of all ranks (strong: the whole dataset once)
    gt_total = int(gt.item())
    value = gt_total * args.steps / elapsed / 1e9
    k_ms = stages["k_encode"] / max(calls, 1)
    alg = rows.line_bytes + out_bytes
    wl = law_name(args.law)
    wkey = "%s/%dx%d" % (wl, S, n)
    if args.mode == "biobank":
        metric = "input GT bytes/sec encoded, 100k-sample x 5M-variant VCF, row-sharded"
        wdesc = ("%s %d samples x %d-variant batch per GPU (BASELINE configs[3]: one batch of the "
                 "5M/N-row shard; batches are independent and run back to back)" % (wl, S, n))
    else:
        metric = "input GT bytes/sec encoded, 2504-sample x 1M-variant VCF"
        if args.scaling == "strong":
            wdesc = "%s %d samples x %d variants split over %d GPU(s) (BASELINE configs[1])" % (wl, S, args.rows, world)
        else:
            wdesc = "%s %d samples x %d variants per GPU (BASELINE configs[1])" % (wl, S, n)
    roof = {"kernel": "k_encode", "bound": "hbm", "achieved": round(alg / (k_ms * 1e-3) / 1e9, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": load_pmc(wkey),
            "step_traffic": load_pmc_step(wkey),
            "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(k_ms, 4),
            "measured_torch_copy_gbs": copy_gbs,
            "stages_ms": {k: round(v / max(calls, 1), 4) for k, v in stages.items()}}
    res = {"metric": metric,
           "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
           "scaling": args.scaling, "vs_baseline": None, "dtype": "u8", "data": "synthetic (generated in HBM)",
           "config": {"workload": wdesc,
                      "samples": S, "rows_per_gpu": n, "gt_bytes_per_gpu": rows.gt_bytes,
                      "line_bytes_per_gpu": rows.line_bytes, "record_bytes_per_gpu": out_bytes,
                      "compression_ratio": round(out_bytes / rows.line_bytes, 4),
                      "deferred_rows": deferred,
                      "parallelism": "row shards x%d, RCCL all-gather of shard sizes" % world},
           "rccl_world": rccl,
           "roofline": roof}
    if rehearsal and args.rows != rows_asked:
        res["config"]["rehearsal_rows_per_rank"] = args.rows
    if world > 1 and args.mode == "encode" and args.scaling == "weak" and not args.no_strong:
        # BASELINE's metric is one fixed 2504 x 1M dataset on 1/2/4/8 GPUs:
        # the same ranks, in the same process group, then time the strong
        # split of the N=1 line's dataset (rank r: rows [1M r/N, 1M (r+1)/N))
        del P, rows, out, rec
        torch.cuda.empty_cache()
        s0, s1 = rows_asked * rank // world, rows_asked * (rank + 1) // world
        ns = s1 - s0
        Q = phase(ns, lambda: workload.DeviceRows(torch, vcfc, ns, S, args.law, seed=1000, device=dev,
                                                  rows_of=(rows_asked, s0)))
        per_rank = gather_ints(torch, dist, cdev, world, [ns, Q["rows"].gt_bytes, int(Q["rec"][ns].item())])
        res["strong"] = strong_summary(per_rank, Q["elapsed"], args.steps,
                                       Q["stages"]["k_encode"] / max(Q["calls"], 1), rows_asked, law_name(args.law))
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
    sys.exit(main() or 0)
