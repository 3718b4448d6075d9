"""Per-launch HBM bytes of the encoder (k_encode_fast + k_encode_var; the
round-2 k_encode_general counted where present) from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE;
separate runs, MI355X_MICROARCH.md's recipe), written as the summary
bench.py's roofline.traffic reads (profiles/pmc_k_encode*.json).  Usage:
  python tools/pmc_encode_json.py <fetch_dir> <write_dir> <workload key> <out.json> <source note>"""
import csv
import json
import sys
from collections import defaultdict

KERNELS = ("k_encode_fast", "k_encode_var", "k_encode_general", "k_encode_defer", "k_compact_out")


def per_kernel(d, counter):
    """Counter total of each kernel per encode call: summed over all its
    dispatches (k_encode_defer<1> and <2>, the compaction and its gated
    second launch) and divided by the calls (one k_encode_fast dispatch each)."""
    tot, calls = defaultdict(float), 0
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split()[-1]
        if r["Counter_Name"] == counter and name in KERNELS:
            tot[name] += float(r["Counter_Value"])
            calls += name == "k_encode_fast"
    return {k: v / max(calls, 1) for k, v in tot.items()}


def main():
    fdir, wdir, key, out, note = sys.argv[1:6]
    f, w = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    kern = {}
    for k in KERNELS:
        fb, wb = int(f.get(k, 0) * 1024 * 2), int(w.get(k, 0) * 1024)
        kern[k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb}
    enc = [k for k in KERNELS if k != "k_compact_out"]
    res = {"workload": key, "kernel": "k_encode (k_encode_fast + k_encode_var + k_encode_defer)", "source": note,
           "fetch_bytes_per_launch": sum(kern[k]["fetch_bytes"] for k in enc),
           "write_bytes_per_launch": sum(kern[k]["write_bytes"] for k in enc),
           "hbm_bytes_per_launch": sum(kern[k]["hbm_bytes"] for k in enc),
           "kernels": kern,
           "correction": "FETCH_SIZE(KiB)*1024*2 (gfx950 half-count of wide coalesced reads), WRITE_SIZE(KiB)*1024"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
