#!/bin/bash
# prof_bench.sh <outdir> [bench args...] : bench.py under rocprofv3 (extra args: e.g. --workload chr1_30x) — kernel-trace stats, then PMC passes
# (FETCH_SIZE, WRITE_SIZE in separate passes, counters only), per MI355X_MICROARCH.md's HBM section.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/${1:-gpurun_out/prof}
shift || true
EXTRA="$*"
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 50 --warmup 5 --reps 3 --no-cpu-baseline --no-parity --many-batches 0 --no-e2e $EXTRA > $OUT/trace.log 2>&1
i=0
for pass in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass -d $OUT/pmc$i -o run --output-format csv -- \
      python3 $ROOT/bench.py --steps 10 --warmup 2 --reps 2 --min-ms 5 --no-cpu-baseline --no-parity --many-batches 0 --no-e2e $EXTRA > $OUT/pmc$i.log 2>&1
done
