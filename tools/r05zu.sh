#!/bin/bash
# r05zu: host worker pool A/B on one box, interleaved (three rounds): the lone process_bam stream and process_bams
# (tools/pbams_trace.py, 6 x 10,000x BAMs) with the pileup library before the pool (pp_old), the pool with a spinning
# waiter (pp_spin) and the pool with a sleeping waiter (in-tree)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zu}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in pp_old pp_spin cur; do
    L=""; [ $v = cur ] || L="tools/pp_ab_run.py $v.so"
    timeout -k 10 300 python3 -u $L tools/pbams_trace.py 6 16 > $OUT/${v}_$r.log 2>&1 || { tail -20 $OUT/${v}_$r.log; exit 1; }
    echo "$v $r $(tail -1 $OUT/${v}_$r.log)"
  done
done
