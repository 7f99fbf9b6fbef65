"""Per-kernel averages of the counters collected by tools/pmc_kernel.sh: pmc_report.py <outdir> [name-substring]"""
import collections
import csv
import os
import sys

src = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "spg::"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(os.listdir(src)):
    f = os.path.join(src, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:40s} {sum(v) / len(v):16.1f}  (n={len(v)})")
