#!/usr/bin/env python3
"""Side-by-side per-kernel averages (us) of kernel-trace A/B runs:
scripts/ab_table.py OUTDIR name1 name2 ... [--top N]"""
import csv
import glob
import re
import sys

args = sys.argv[1:]
top = 34
if "--top" in args:
    i = args.index("--top")
    top = int(args[i + 1])
    del args[i:i + 2]
out, names = args[0], args[1:]
data = {}
for n in names:
    f = glob.glob(f"{out}/ab/{n}/*kernel_stats.csv")
    if not f:
        continue
    d = {}
    for r in csv.DictReader(open(f[0])):
        m = re.search(r"(k_[a-z_0-9]+(<[^>(]*>)?)", r["Name"])
        if m:
            d[m.group(1)] = float(r["AverageNs"]) / 1e3
    data[n] = d
keys = sorted(set().union(*[d.keys() for d in data.values()]),
              key=lambda k: -max(d.get(k, 0) for d in data.values()))
print(f'{"kernel":45s}' + "".join(f"{n:>9s}" for n in data))
for k in keys[:top]:
    print(f"{k[:45]:45s}" + "".join(f"{data[n].get(k, 0):9.1f}" for n in data))
