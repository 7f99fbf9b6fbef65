#!/bin/bash
# r05zc: replay-walk prefetch A/B (nopf = -DSPG_REPLAY_NOPF) on the parity-mode and uncapped sars10k lines, interleaved
# (two rounds), then the wave timeline of the default build
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zc}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
B="bench.py --legs parity --no-cpu-baseline --reps 10"
for r in 1 2; do
  timeout -k 10 200 python3 -u $B > $OUT/base_$r.json 2> $OUT/base_$r.err || { tail -5 $OUT/base_$r.err; exit 1; }
  timeout -k 10 200 python3 -u tools/ab_run.py nopf.so $B > $OUT/nopf_$r.json 2> $OUT/nopf_$r.err || { tail -5 $OUT/nopf_$r.err; exit 1; }
done
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*_?.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    p = d.get("parity_mode", {})
    r, pr = d["roofline"], p.get("roofline", {})
    print(f.split("/")[-1], "main step %.4f kernel %.4f ms frac %.4f replays %s" % (d["ms_per_step"], r["kernel_ms"], r["frac"], d.get("replayed_positions_per_gpu_step")),
          "| parity step %.4f kernel %.4f ms frac %.4f replays %s" % (p["ms_per_step"], pr["kernel_ms"], pr["frac"], p.get("replayed_positions_per_gpu_step")))
PY
bash tools/r05zb.sh ${1:-r05zc}/wt
