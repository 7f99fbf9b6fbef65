#!/bin/bash
# r05zk: the fused finalize's memory round trips — interleaved A/B (two rounds) on the sars10k main + parity lines of
# base (split tail, finalize after the record stores, parameters and 10^-k table from memory), fin1 (finalize on the
# LDS images before the stores), fin1lds (+ parameters from an LDS copy), fin1ldsx (+ P from exp10), lds0 (LDS
# parameters + exp10, stores first), nosplit (the r05 launch); then each variant's parity-mode wave timeline
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zk}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
B="bench.py --legs parity --no-cpu-baseline --reps 10"
V="fin1 fin1lds fin1ldsx lds0 nosplit"
for r in 1 2; do
  timeout -k 10 200 python3 -u $B > $OUT/base_$r.json 2> $OUT/base_$r.err || { tail -5 $OUT/base_$r.err; exit 1; }
  for v in $V; do
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
timeout -k 10 300 python3 -u tools/wavetimes.py 10000 $OUT/wt_base.json 8000 > $OUT/wt_base.log 2>&1 || { tail -20 $OUT/wt_base.log; exit 1; }
for v in $V; do
  timeout -k 10 300 python3 -u tools/ab_run.py $v.so tools/wavetimes.py 10000 $OUT/wt_$v.json 8000 > $OUT/wt_$v.log 2>&1 || { tail -20 $OUT/wt_$v.log; exit 1; }
done
python3 - $OUT <<'PY'
import json, sys
for v in "base fin1 fin1lds fin1ldsx lds0 nosplit".split():
    d = json.load(open(f"{sys.argv[1]}/wt_{v}.json"))
    print(v, "span", d["span_us"], "finalize_us", d["finalize_us_of_those"])
    for w in d["last_10_waves_to_end"][:3]: print("   last", w)
PY
