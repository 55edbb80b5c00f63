"""Per-kernel average durations (us) of scripts/kt_variants.sh runs."""
import csv
import glob
import sys

KEYS = ["k_bucket_fill1<float, 0", "k_bucket_fill2<float, 0",
        "k_bucket_fill1<float, 1", "k_bucket_fill2<float, 1",
        "k_bucket_count<float, 0", "k_bucket_count<float, 1",
        "k_scan_columns", "k_scan_bins", "k_scatter_tab", "k_scatter_pad", "k_gather_tab"]
out = sys.argv[1]
for n in sys.argv[2:]:
    fs = glob.glob(f"{out}/{n}/**/*kernel_stats.csv", recursive=True)
    if not fs:
        print(n, "missing")
        continue
    d = {r["Name"]: float(r["AverageNs"]) / 1e3
         for r in csv.DictReader(open(fs[0]))}
    print(n, {k.replace("k_bucket_", ""): round(sum(v for kk, v in d.items()
                                                     if k in kk), 1)
              for k in KEYS})
