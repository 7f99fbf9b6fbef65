#!/bin/bash
# r05zb: the deep kernel's per-wave timeline (chunk-loop end and fused-finalize flag per wave), uncapped and parity mode
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zb}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
for t in "uncapped 0" "parity 8000"; do
  set -- $t
  timeout -k 10 300 python3 -u tools/wavetimes.py 10000 $OUT/wt_$1.json $2 > $OUT/wt_$1.log 2>&1 || { tail -20 $OUT/wt_$1.log; exit 1; }
done
python3 - $OUT <<'PY'
import json, sys
for t in ("uncapped", "parity"):
    d = json.load(open(f"{sys.argv[1]}/wt_{t}.json"))
    print(t, {k: d[k] for k in ("waves", "G", "span_us", "busy_wave_us_over_span", "fused_finalize_waves")})
    print("  finalize_us", d["finalize_us_of_those"], "\n  loop_us_of_those", d["loop_us_of_those"], "\n  loop_us_all", d["loop_us_all"])
    for w in d["last_10_waves_to_end"][:6]: print("  last", w)
    for w in d["longest_waves"][:6]: print("  long", w)
PY
