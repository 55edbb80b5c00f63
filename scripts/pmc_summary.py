"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel per pass."""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
data = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "pass*", "*counter_collection.csv"))):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row["Kernel_Name"]
            m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", name)
            short = m.group(1) if m else name.split("(")[0][-60:]
            data[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, ctr in data.items():
    print("==", k)
    for c, vals in sorted(ctr.items()):
        print(f"   {c:28s} {sum(vals)/len(vals):16.4g}  (n={len(vals)})")
