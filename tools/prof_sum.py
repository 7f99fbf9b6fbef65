"""prof_sum.py <dir>: top kernels of every rocprofv3 kernel_stats.csv under <dir>, and FETCH/WRITE per dispatch of the device
pileup kernels and the deep kernel from the counter CSVs (dev tool)."""
import csv, glob, os, sys, collections
OUT = sys.argv[1]
for f in sorted(glob.glob(os.path.join(OUT, '**', '*kernel_stats.csv'), recursive=True)):
    print('==', os.path.relpath(f, OUT))
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r.get('TotalDurationNs', 0)))
    for r in rows[:12]:
        print(f"  {r['Name'][:70]:70s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:10.1f} us  total {float(r['TotalDurationNs'])/1e6:9.2f} ms")
for f in sorted(glob.glob(os.path.join(OUT, '**', '*counter_collection.csv'), recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r.get('Kernel_Name', '')
        for key in ('k_inflate_par', 'k_inflate(', 'k_pileup_fill', 'k_tile_first', 'k_acc_seg<4', 'k_fill(', 'k_fill<',
                    'k_fill_starts', 'k_f2_fill', 'k_f2_count', 'k_f2_base', 'k_crc32', 'k_bam_'):
            if key in k:
                acc[(key, r['Counter_Name'])][r['Dispatch_Id']] += float(r['Counter_Value'])
    print('==', os.path.relpath(f, OUT))
    for (k, c), d in sorted(acc.items()):
        m = sum(d.values()) / len(d)
        corr = f" (x2 gfx950 correction: {2 * m:.4g})" if c.startswith("FETCH") else ""
        print(f"  {k:16s} {c:12s} mean per dispatch {m:.4g} KB{corr} dispatches {len(d)}")
