#!/usr/bin/env python3
"""Means per library of tools/ab.sh records: python tools/ab_summary.py <ab.txt>..."""
import collections
import sys

for path in sys.argv[1:]:
    d = collections.OrderedDict()
    for line in open(path):
        p = line.split()
        if len(p) < 5:
            continue
        d.setdefault(p[0], []).append((float(p[2]), float(p[3]), float(p[4])))
    print(path, " | ".join("%s k=%.3f c=%.3f s=%.3f" % (k, *(sum(x[i] for x in v) / len(v) for i in range(3)))
                           for k, v in d.items()))
