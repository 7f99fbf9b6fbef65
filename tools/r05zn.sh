#!/bin/bash
# r05zn: the fused finalize with no memory round trip but its candidate slot — parameters from a workgroup LDS copy and
# P = exp10(-k) eps(r) (ldsx), also run before the record stores (fin1ldsx): parity-mode wave timelines of diagnostic
# builds (per-stage times of the fused-finalize waves) and interleaved A/B of the sars10k main + parity lines
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zn}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
for v in diagwt d_ldsx d_fin1ldsx; do
  SPG_WAVE_TIMES=/tmp/wt_$v.bin timeout -k 10 300 python3 -u tools/ab_run.py $v.so tools/wavetimes.py 10000 $OUT/wt_$v.json 8000 > $OUT/wt_$v.log 2>&1 || { tail -20 $OUT/wt_$v.log; exit 1; }
  cp /tmp/wt_$v.bin $OUT/
done
python3 - $OUT <<'PY'
import json, sys
import numpy as np
o = sys.argv[1]
q = lambda a: {p: round(float(np.percentile(a, p)), 2) for p in (5, 50, 95)}
for v in "diagwt d_ldsx d_fin1ldsx".split():
    d = json.load(open(f"{o}/wt_{v}.json"))
    print(v, "span", d["span_us"], "finalize_us", d["finalize_us_of_those"])
    for w in d["last_10_waves_to_end"][:2]: print("   last", w)
    raw = open(f"{o}/wt_{v}.bin", "rb").read()
    at, last = 0, None
    while at < len(raw):
        n, g = np.frombuffer(raw[at:at + 16], np.int64); at += 16
        last = np.frombuffer(raw[at:at + 16 * n], np.uint32).reshape(n, 4); at += 16 * int(n)
    w = last[last[:, 2] != 0]
    lend = (w[:, 1] >> 15) * 10e-3; life = (w[:, 2] & 0xFFFFF) * 10e-3; fin = (w[:, 3] & 0xFFFFF) * 10e-3
    t = ((w[:, 3] >> 20) & 1).astype(bool)
    print("   fused waves: loop end -> mark", q(fin[t] - lend[t]), "mark -> end", q(life[t] - fin[t]))
    print("   other waves: loop end -> mark", q(fin[~t] - lend[~t]), "mark -> end", q(life[~t] - fin[~t]))
PY
B="bench.py --legs parity --no-cpu-baseline --reps 10"
for r in 1 2; do
  timeout -k 10 200 python3 -u $B > $OUT/base_$r.json 2> $OUT/base_$r.err || { tail -5 $OUT/base_$r.err; exit 1; }
  for v in ldsx fin1ldsx; do
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
