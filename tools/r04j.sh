# r04j: k_count_cols (lone mid-depth batch) parity tests, then the sars1k leg A/B (count path vs the fused list mode)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04j}; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "mid_depth or calls_only or fused or sars or bq or multibatch or shallow_then" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for m in 1 0; do
  SPG_COUNT_COLS=$( [ $m = 1 ] && echo -1 || echo 0 ) timeout -k 10 300 python3 -u bench.py --no-main --legs sars1k --reps 5 --no-cpu-baseline > $OUT/sars1k_$m.json 2> $OUT/sars1k_$m.err || { echo "bench $m failed"; tail -20 $OUT/sars1k_$m.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/sars1k_$m.json').read().strip().splitlines()[-1]); s=d['sars1k']; print('$m', s['ms_per_step'], s['roofline']['frac'], s['roofline']['kernel'])"
done
