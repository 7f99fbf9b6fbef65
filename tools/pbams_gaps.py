"""pbams_gaps.py <trace dir> <marks.json>: GPU busy time (union of kernel and memory-copy intervals, rocprofv3 CSVs)
inside each marked window of tools/pbams_trace.py, the longest idle gaps, and per-kernel time inside it (dev tool)."""
import csv
import glob
import json
import os
import sys

d, mk = sys.argv[1], json.load(open(sys.argv[2]))
iv = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60]))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r.get("Direction", r.get("Operation", "copy"))))
iv.sort()
for name, m in mk.items():
    a, b = m["ns"]
    sel = [(max(s, a), min(e, b), k) for s, e, k in iv if e > a and s < b]
    busy, cur_s, cur_e, gaps, last = 0, None, None, [], a
    per = {}
    for s, e, k in sel:
        per[k] = per.get(k, 0) + (e - s)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            gaps.append((s - (cur_e if cur_e is not None else a), cur_e if cur_e is not None else a))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
        gaps.append((b - cur_e, cur_e))
    w = b - a
    print(f"== {name}: window {w / 1e6:.2f} ms, GPU busy (kernels + copies, union) {busy / 1e6:.2f} ms = {100 * busy / w:.1f} %")
    for g, at in sorted(gaps, reverse=True)[:8]:
        print(f"   idle {g / 1e6:7.3f} ms at +{(at - a) / 1e6:8.3f} ms")
    for k, t in sorted(per.items(), key=lambda x: -x[1])[:14]:
        print(f"   {t / 1e6:8.3f} ms  {k}")
