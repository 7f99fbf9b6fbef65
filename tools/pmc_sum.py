"""pmc_sum.py <dir> <kernel substring>: mean per dispatch of every counter in the rocprofv3 --pmc CSVs under <dir>,
one line per (variant dir, counter).  Dev tool."""
import csv
import glob
import os
import sys
from collections import defaultdict

root, kname = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    acc = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        if kname in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    tag = os.path.relpath(f, root).split(os.sep)[0]
    for c, d in sorted(acc.items()):
        print(f"{tag:14s} {c:28s} {sum(d.values()) / len(d):.4g}  (dispatches {len(d)})")
