#!/bin/bash
# prof_many.sh <outdir> [bench args...]: kernel-trace stats of a bench workload (default config 4 with
# 2,000 BAMs), then FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, counters only).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/${1:-gpurun_out/prof_many}
shift || true
ARGS=${@:-"--workload sars_many --many-batches 2000 --reps 3 --warmup 2"}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 $ROOT/bench.py $ARGS > $OUT/trace.log 2>&1
i=0
for pass in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass -d $OUT/pmc$i -o run --output-format csv -- \
      python3 $ROOT/bench.py $ARGS > $OUT/pmc$i.log 2>&1
done
