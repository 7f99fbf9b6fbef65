# r04k: sars1k under rocprof (count path on / off), and sars1k after the parity leg (the default bench's order)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04k}; mkdir -p $OUT
cd /tmp
for m in -1 0; do
  SPG_COUNT_COLS=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$m -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-main --legs sars1k --reps 3 --no-cpu-baseline > $OUT/p_$m.json 2> $OUT/p_$m.err || { echo "prof $m failed"; tail -20 $OUT/p_$m.err; exit 1; }
done
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u bench.py --no-main --legs parity,sars1k --reps 5 --no-cpu-baseline > $OUT/ps.json 2> $OUT/ps.err || { echo "ps failed"; tail -20 $OUT/ps.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/ps.json').read().strip().splitlines()[-1]); print(d['sars1k']['ms_per_step'], d['sars1k']['roofline']['kernel_ms'])"
find $OUT -name "*kernel_stats.csv" | while read f; do echo $f; head -8 $f | cut -c1-200; done
