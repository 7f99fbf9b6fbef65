#!/bin/bash
# r05x: k_f2_fill A/B (tools/build_ab.sh variants f2u2 / f2u4 vs the default build): rocprof kernel stats of the e2e leg
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/r05x
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
for rep in 1 2; do
  for v in default f2u2 f2u4; do
    if [ $v = default ]; then cmd="$ROOT/tools/e2e_only.py 2 0 16"; else cmd="$ROOT/tools/ab_run.py $v.so $ROOT/tools/e2e_only.py 2 0 16"; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${v}_$rep -o run --output-format csv -- python3 $cmd > $OUT/${v}_$rep.log 2>&1 || { echo "$v failed"; tail -5 $OUT/${v}_$rep.log; exit 1; }
    python3 - $OUT/${v}_$rep/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_f2_fill" in r["Name"] or "k_inflate_par" in r["Name"]:
        print(sys.argv[2], r["Name"][:20], "avg %.1f us" % (float(r["AverageNs"]) / 1e3), "calls", r["Calls"])
PY
  done
done
find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete
