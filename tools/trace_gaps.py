#!/usr/bin/env python3
"""One step of a rocprofv3 kernel trace with the idle gaps between kernels:
   python tools/trace_gaps.py <kernel_trace.csv> <first-kernel substring> [nth]
The step runs from the nth-to-last launch whose name holds the substring to
the next such launch (default: the second-to-last step of the run)."""
import csv
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    nth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
    i0, i1 = idx[-nth], idx[-nth + 1]
    t0 = int(rows[i0]["Start_Timestamp"])
    prev = None
    busy = gaps = 0.0
    print("%9s %9s %8s  %s" % ("start_us", "dur_us", "gap_us", "kernel"))
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        g = (s - prev) / 1e3 if prev is not None else 0.0
        busy += (e - s) / 1e3
        gaps += max(g, 0.0)
        print("%9.1f %9.1f %8.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, g, r["Kernel_Name"][:80]))
        prev = e
    end = int(rows[i1]["Start_Timestamp"])
    print("step %.1f us: kernels %.1f us, gaps %.1f us" % ((end - t0) / 1e3, busy, gaps))


if __name__ == "__main__":
    main()
