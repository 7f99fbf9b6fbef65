"""Per-kernel SQ counter averages of a tools/tile_ab.sh run: sq_report.py <outdir> [substring ...]
Prints per-dispatch averages and, with --per N, per-unit values (N units per dispatch)."""
import collections
import csv
import os
import sys

base = sys.argv[1]
subs = [a for a in sys.argv[2:] if not a.startswith("--")] or ["k_acc_tile", "k_acc_one"]
for d in sorted(os.listdir(base)):
    f = os.path.join(base, d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        if any(s in r["Kernel_Name"] for s in subs):
            agg[r["Kernel_Name"][:34]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        print(d, k, " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))
