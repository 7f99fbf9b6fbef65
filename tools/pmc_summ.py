"""Print per-variant average PMC counters of the deep accumulate kernel (tools/pmc_ab.sh output)."""
import csv, glob, collections, sys, os
root = sys.argv[1]
for v in sorted(os.listdir(root)):
    if not os.path.isdir(os.path.join(root, v)):
        continue
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, v, 'p*', 'run_counter_collection.csv')):
        for r in csv.DictReader(open(f)):
            if 'k_acc_seg' in r['Kernel_Name']:
                agg[r['Counter_Name']].append(float(r['Counter_Value']))
    print(v, ' '.join(f"{c}={sum(x)/len(x):.4g}" for c, x in sorted(agg.items())))
