#!/usr/bin/env python3
"""Kernel statistics (calls, total, average, share) from a rocprofv3 rocpd
SQLite database, as CSV -- the equivalent of rocprofv3 --stats.

  python scripts/rocpd_stats.py gpurun_out/prof/x_results.db > out.csv
"""
import collections
import csv
import sqlite3
import sys


def main(path):
    con = sqlite3.connect(path)
    rows = con.execute(
        "select ks.kernel_name, kd.start, kd.end from rocpd_kernel_dispatch kd"
        " join rocpd_info_kernel_symbol ks on kd.kernel_id = ks.id").fetchall()
    agg = collections.defaultdict(lambda: [0, 0])
    for name, s, e in rows:
        a = agg[name]
        a[0] += 1
        a[1] += e - s
    total = sum(v[1] for v in agg.values()) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for name, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        w.writerow([name, c, t, t // c, f"{100.0 * t / total:.4f}"])


if __name__ == "__main__":
    main(sys.argv[1])
