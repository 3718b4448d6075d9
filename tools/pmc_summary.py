"""Summarise rocprofv3 --pmc counter CSVs (one directory per pass) per kernel:
mean counter value per dispatch and mean duration.  Usage:
  python tools/pmc_summary.py gpurun_out/<tag>  [kernel-substring]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(root, ksub=None):
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(root, "pmc*", "run_counter_collection.csv")):
        seen = set()
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            if ksub and ksub not in name:
                continue
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (f, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {}
    for k, cs in vals.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["dispatch_ms"] = sum(dur[k]) / len(dur[k])
    return out


if __name__ == "__main__":
    res = load(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
    print(json.dumps(res, indent=1, sort_keys=True))
