#!/bin/bash
# r05zd: fused finalize parameters through scalar loads A/B (sparam = -DSPG_FUSE_SPARAM=1) on the parity-mode and uncapped sars10k lines, interleaved
# (two rounds), then the wave timeline of the default build
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zd}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
B="bench.py --legs parity --no-cpu-baseline --reps 10"
for r in 1 2; do
  timeout -k 10 200 python3 -u $B > $OUT/base_$r.json 2> $OUT/base_$r.err || { tail -5 $OUT/base_$r.err; exit 1; }
  timeout -k 10 200 python3 -u tools/ab_run.py sparam.so $B > $OUT/sparam_$r.json 2> $OUT/sparam_$r.err || { tail -5 $OUT/sparam_$r.err; exit 1; }
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
bash tools/r05zb.sh ${1:-r05zd}/wt
SPG_WAVE_TIMES=/tmp/wt_sparam.bin timeout -k 10 300 python3 -u tools/ab_run.py sparam.so tools/wavetimes.py 10000 $OUT/wt_sparam_parity.json 8000 > $OUT/wt_sparam.log 2>&1 || { tail -20 $OUT/wt_sparam.log; exit 1; }
python3 -c "
import json,sys; d=json.load(open('$OUT/wt_sparam_parity.json')); print('sparam parity span', d['span_us'], 'finalize', d['finalize_us_of_those']); print(d['last_10_waves_to_end'][:3])"
