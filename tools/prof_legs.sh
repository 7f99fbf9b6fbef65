#!/bin/bash
# prof_legs.sh <outdir> <leg>... : per bench leg, rocprofv3 --kernel-trace --stats over bench.py restricted to that leg, then
# the PMC passes FETCH_SIZE and WRITE_SIZE (separate runs, counters only; MI355X_MICROARCH.md HBM section).
# Legs: main parity sars1k sars100k sars100k_capped config4 chr1.  tools/summarize_prof.py turns each into profiles/.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/$1
shift
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
for leg in "$@"; do
  case $leg in
    main) A="--legs none" ;;
    config4) A="--no-main --legs config4 --many-batches 0 --per-bam-bams 2000" ;;
    *) A="--no-main --legs $leg" ;;
  esac
  D=$OUT/$leg
  mkdir -p $D
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- \
      python3 $ROOT/bench.py --steps 20 --warmup 3 --reps 3 $A > $D/trace.json 2> $D/trace.err || { echo "$leg trace failed"; tail -5 $D/trace.err; exit 1; }
  i=0
  for pass in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 400 rocprofv3 --pmc $pass -d $D/pmc$i -o run --output-format csv -- \
        python3 $ROOT/bench.py --steps 5 --warmup 1 --reps 2 --min-ms 5 $A > $D/pmc$i.json 2> $D/pmc$i.err || { echo "$leg pmc $pass failed"; tail -5 $D/pmc$i.err; exit 1; }
  done
  echo "$leg ok"
done
