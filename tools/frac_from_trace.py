"""Recompute a bench line's roofline fraction from a committed rocprofv3
kernel trace of the same process (tools/gpu_check.sh profbench: the bench
command itself under `rocprofv3 --kernel-trace --stats`).

usage: python tools/frac_from_trace.py profiles/r05/final/bench_under_prof.json \
           profiles/r05/final/kernel_trace.csv

The encoder launch is k_encode_fast + k_encode_var + k_encode_defer (the
bench line's `k_encode` stage).  Per kernel: the mean dispatch duration over
all launches and over the timed ones (the first `warmup` launches dropped);
then algorithmic bytes / summed mean / peak against the line's own frac.
"""
import collections
import csv
import json
import sys

ENCODER = ("k_encode_fast", "k_encode_var", "k_encode_defer")


def main(line_path, trace_path):
    line = json.load(open(line_path))
    roof = line["roofline"]
    warm = int(line["warmup"])
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(trace_path)):
        name = r["Kernel_Name"]
        key = name.split("::")[1].split("(")[0] if "::" in name else name
        dur[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot_all = tot_timed = 0.0
    for k, v in sorted(dur.items()):
        if not k.startswith(ENCODER):
            continue
        timed = v[warm:] if len(v) > warm else v
        a, t = sum(v) / len(v) / 1e6, sum(timed) / len(timed) / 1e6
        tot_all += a
        tot_timed += t
        print("%-24s launches %3d  mean %.4f ms  timed mean %.4f ms" % (k, len(v), a, t))
    b = roof["algorithmic_bytes_per_launch"]
    for label, ms in (("all launches", tot_all), ("timed launches", tot_timed)):
        frac = b / (ms * 1e6) / roof["peak"]
        print("%-15s %.4f ms  %.1f GB/s  frac %.4f  (line: %.4f ms, frac %.4f; %+.2f %%)"
              % (label, ms, b / (ms * 1e6), frac, roof["avg_launch_ms"], roof["frac"],
                 100.0 * (frac / roof["frac"] - 1.0)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
