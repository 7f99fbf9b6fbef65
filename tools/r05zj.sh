#!/bin/bash
# r05zj: fused deep launch with split tail columns — parity tests of the fused path, then interleaved A/B on the
# sars10k main and parity-mode lines (base = split 1024 columns after a 4,096-wave G/2 tail; nosplit = the r05 launch;
# split2k = 2,048 split columns; notail = split columns only), two rounds, then the wave timeline of the default build
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zj}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/parity_tests.log 2>&1 || { tail -30 $OUT/parity_tests.log; exit 1; }
tail -3 $OUT/parity_tests.log
B="bench.py --legs parity --no-cpu-baseline --reps 10"
for r in 1 2; do
  timeout -k 10 200 python3 -u $B > $OUT/base_$r.json 2> $OUT/base_$r.err || { tail -5 $OUT/base_$r.err; exit 1; }
  for v in nosplit split2k notail; do
    timeout -k 10 200 python3 -u tools/ab_run.py $v.so $B > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { tail -5 $OUT/${v}_$r.err; exit 1; }
  done
done
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*_?.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    p = d.get("parity_mode", {})
    r, pr = d["roofline"], p.get("roofline", {})
    print(f.split("/")[-1], "main step %.4f kernel %.4f ms frac %.4f" % (d["ms_per_step"], r["kernel_ms"], r["frac"]),
          "| parity step %.4f kernel %.4f ms frac %.4f" % (p["ms_per_step"], pr["kernel_ms"], pr["frac"]))
PY
bash tools/r05zb.sh ${1:-r05zj}/wt
