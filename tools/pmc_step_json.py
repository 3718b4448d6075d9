"""HBM bytes per step of a multi-kernel path (bench.py --mode devfile: the
line index, placement, encoder and compaction of one vcfc_compress_device
call) from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs,
MI355X_MICROARCH.md's recipe).  Every dispatch from the first line-index
kernel on is counted except torch's own kernels (the output check) and the
generator; the sum is divided by the number of calls (warmup + steps), and
written as the summary bench.py's roofline.traffic reads
(profiles/pmc_devfile*.json).  Usage:
  python tools/pmc_step_json.py <fetch_dir> <write_dir> <calls> <workload key> <out.json> <source note>
                                [first kernels, comma-separated (default: the line-index kernels)] [step name]
(bench.py --mode query: first kernel k_query_match -> profiles/pmc_k_query.json)"""
import csv
import json
import sys
from collections import defaultdict

FIRST = ("k_nl_hop", "k_nl_count", "k_nl_scan")   # the step's first kernel (hop or scan index)


def per_kernel(d, counter, first=FIRST):
    rows = []
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        rows.append((int(r["Dispatch_Id"]), name, float(r["Counter_Value"])))
    rows.sort()
    start = min((i for i, n, _ in rows if n.split("<")[0].split()[-1] in first), default=None)
    if start is None:
        raise SystemExit("no %s kernel in %s" % ("/".join(first), d))
    tot = defaultdict(float)
    for i, n, v in rows:
        if i >= start and "at::" not in n and n != "k_synth":
            tot[n] += v
    return tot


def main():
    fdir, wdir, calls, key, out, note = sys.argv[1:7]
    first = tuple(sys.argv[7].split(",")) if len(sys.argv) > 7 else FIRST
    step = sys.argv[8] if len(sys.argv) > 8 else "vcfc_compress_device step (all kernels of one call)"
    calls = int(calls)
    f, w = per_kernel(fdir, "FETCH_SIZE", first), per_kernel(wdir, "WRITE_SIZE", first)
    kern = {}
    for k in sorted(set(f) | set(w)):
        fb, wb = int(f.get(k, 0) * 1024 * 2 / calls), int(w.get(k, 0) * 1024 / calls)
        kern[k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb}
    res = {"workload": key, "kernel": step, "source": note,
           "calls": calls,
           "fetch_bytes_per_launch": sum(v["fetch_bytes"] for v in kern.values()),
           "write_bytes_per_launch": sum(v["write_bytes"] for v in kern.values()),
           "hbm_bytes_per_launch": sum(v["hbm_bytes"] for v in kern.values()),
           "kernels": kern,
           "correction": "FETCH_SIZE(KiB)*1024*2 (gfx950 half-count of wide coalesced reads), WRITE_SIZE(KiB)*1024"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
