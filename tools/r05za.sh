#!/bin/bash
# r05za: the deep kernel's per-wave timeline uncapped and in parity mode (max_depth 8000; tools/wavetimes.py), then
# FETCH_SIZE / WRITE_SIZE per dispatch of the e2e device-path kernels (k_inflate_par, k_f2_*, k_bam_*), one pass each
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05za}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/wavetimes.py 10000 $OUT/wt_uncapped.json 0 > $OUT/wt_uncapped.log 2>&1 || { tail -20 $OUT/wt_uncapped.log; exit 1; }
timeout -k 10 300 python3 -u tools/wavetimes.py 10000 $OUT/wt_parity.json 8000 > $OUT/wt_parity.log 2>&1 || { tail -20 $OUT/wt_parity.log; exit 1; }
cd /tmp
i=0
for pass in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass -d $OUT/e2e_pmc$i -o run --output-format csv -- \
      python3 $ROOT/tools/e2e_only.py 2 0 16 > $OUT/e2e_pmc$i.log 2>&1 || { echo "e2e pmc $pass failed"; tail -20 $OUT/e2e_pmc$i.log; exit 1; }
done
python3 $ROOT/tools/prof_sum.py $OUT > $OUT/summary.txt 2>&1
find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete
find $OUT -name "*.log" -size +1M -delete
cat $OUT/summary.txt
python3 - $OUT <<'PY'
import json, sys
for t in ("uncapped", "parity"):
    d = json.load(open(f"{sys.argv[1]}/wt_{t}.json"))
    print(t, {k: d[k] for k in ("waves", "G", "span_us", "busy_wave_us_over_span", "workgroup_slack_over_wave_time",
                                 "slot_gap_total_over_wave_time", "waves_starting_after_span_minus_10us")})
    print("  life", d["life_us"], "prologue", d["prologue_us"])
    print("  resident", d["resident_waves_over_time"])
PY
