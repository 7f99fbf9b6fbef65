"""Summarise a tools/prof_bench.sh run into profiles/ (tracked): kernel-trace stats + PMC HBM bytes.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE counts half the bytes of wide
coalesced streaming reads (MI355X_MICROARCH.md, HBM section), so it is doubled; WRITE_SIZE is taken
as is.  Writes <tag>_kernel_stats.csv, <tag>_pmc.json and <tag>_summary.md."""
import csv
import collections
import json
import os
import shutil
import sys


def main(src, tag, entries=None, dst="profiles", cmd="bench.py --steps 50 --warmup 5"):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not p.startswith("pmc") or not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            pmc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = {"grid": int(r["Grid_Size"]), "workgroup": int(r["Workgroup_Size"]), "lds": int(r["LDS_Block_Size"]),
                       "vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]), "scratch": int(r["Scratch_Size"])}
    out = {}
    for k, cs in pmc.items():
        if not k.startswith("void spg::") and not k.startswith("spg::"):
            continue
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        rec = dict(meta[k])
        if "FETCH_SIZE" in d:
            rec["read_bytes_per_launch"] = d["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in d:
            rec["write_bytes_per_launch"] = d["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            rec["hbm_bytes_per_launch"] = rec["read_bytes_per_launch"] + rec["write_bytes_per_launch"]
        rec["dispatches"] = max(len(v) for v in cs.values())
        if entries:
            rec["entries"] = int(entries)       # pileup entries per launch of the profiled workload
        out[k.split("(")[0].replace("void ", "")] = rec
    json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    with open(os.path.join(dst, f"{tag}_summary.md"), "w") as f:
        f.write(f"# {tag}: rocprofv3 summary of `bench.py` (1x MI355X)\n\n")
        f.write(f"Kernel trace (`rocprofv3 --kernel-trace --stats`, {cmd}):\n\n")
        f.write("| kernel | calls | avg us | min us | max us | % |\n|---|---|---|---|---|---|\n")
        for r in stats:
            f.write(f"| `{r['Name'].split('(')[0]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                    f"{float(r['MinNs'])/1e3:.1f} | {float(r['MaxNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |\n")
        f.write("\nPMC (separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes of the same command, fewer steps; "
                "FETCH_SIZE x2 per the gfx950 correction):\n\n")
        f.write("| kernel | read MB/launch | write MB/launch | VGPR | LDS B | scratch |\n|---|---|---|---|---|---|\n")
        for k, r in out.items():
            f.write(f"| `{k}` | {r.get('read_bytes_per_launch', 0)/1e6:.1f} | {r.get('write_bytes_per_launch', 0)/1e6:.1f} | "
                    f"{r['vgpr']} | {r['lds']} | {r['scratch']} |\n")
    print(open(os.path.join(dst, f"{tag}_summary.md")).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None,
         sys.argv[4] if len(sys.argv) > 4 else "profiles", sys.argv[5] if len(sys.argv) > 5 else "bench.py --steps 50 --warmup 5")
