"""prof_filter.py <dir>...: keep only the spg:: kernels' rows of rocprofv3 CSVs under each dir (the bench's torch
data generation launches thousands of kernels) and drop the per-dispatch trace, so the profile travels back small."""
import csv
import os
import sys

for root in sys.argv[1:]:
    for dp, _, fs in os.walk(root):
        for f in fs:
            p = os.path.join(dp, f)
            if f == "run_kernel_trace.csv":
                os.remove(p)
            elif f == "run_counter_collection.csv":
                rows = list(csv.reader(open(p)))
                if not rows:
                    continue
                k = rows[0].index("Kernel_Name")
                with open(p, "w", newline="") as o:
                    w = csv.writer(o)
                    w.writerow(rows[0])
                    w.writerows(r for r in rows[1:] if "spg::" in r[k])
