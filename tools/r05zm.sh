#!/bin/bash
# r05zm: where a calling column's wave spends the time after its chunk loop.  Parity-mode sars10k wave timelines (run
# in-process, so an A/B build is the one timed) of the default build, nofin (no finalize: timing only) and diagwt (the
# record's hw-id field holds entry -> end of drain + assemble + record stores); per-stage times of the fused-finalize
# waves vs the others
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zm}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
for v in base nofin diagwt fin1 priofin; do
  L=""; [ $v = base ] || L="tools/ab_run.py $v.so"
  SPG_WAVE_TIMES=/tmp/wt_$v.bin timeout -k 10 300 python3 -u $L tools/wavetimes.py 10000 $OUT/wt_$v.json 8000 > $OUT/wt_$v.log 2>&1 || { tail -20 $OUT/wt_$v.log; exit 1; }
  cp /tmp/wt_$v.bin $OUT/
done
python3 - $OUT <<'PY'
import json, sys
import numpy as np
o = sys.argv[1]
for v in "base nofin diagwt fin1 priofin".split():
    d = json.load(open(f"{o}/wt_{v}.json"))
    print(v, "span", d["span_us"], "finalize_us", d["finalize_us_of_those"])
    for w in d["last_10_waves_to_end"][:2]: print("   last", w)
raw = open(f"{o}/wt_diagwt.bin", "rb").read()
at, last = 0, None
while at < len(raw):
    n, g = np.frombuffer(raw[at:at + 16], np.int64); at += 16
    last = np.frombuffer(raw[at:at + 16 * n], np.uint32).reshape(n, 4); at += 16 * int(n)
w = last[last[:, 2] != 0]
lend = (w[:, 1] >> 15) * 10e-3; life = (w[:, 2] & 0xFFFFF) * 10e-3; fin = (w[:, 3] & 0xFFFFF) * 10e-3
tailed = ((w[:, 3] >> 20) & 1).astype(bool)
q = lambda a: {p: round(float(np.percentile(a, p)), 2) for p in (5, 50, 95)}
print("diagwt fused waves: finish after loop", q(fin[tailed] - lend[tailed]), "finalize after finish", q(life[tailed] - fin[tailed]))
print("diagwt other waves: finish after loop", q(fin[~tailed] - lend[~tailed]), "after finish", q(life[~tailed] - fin[~tailed]))
PY
