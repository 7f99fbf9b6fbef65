#!/bin/bash
# e2e_ab.sh: the end-to-end bench leg with and without the host pileup's page pre-touch (SPP_PRETOUCH), two rounds
OUT=gpurun_out/r03q
mkdir -p $OUT
B="bench.py --no-parity --many-batches 0 --no-chr1 --runs-batches 0 --no-cpu-baseline --reps 3"
for r in 1 2; do
  SPP_PRETOUCH=0 timeout -k 10 300 python3 -u $B > $OUT/nopt_$r.json 2> $OUT/nopt_$r.err || exit 1
  SPP_PRETOUCH=1 timeout -k 10 300 python3 -u $B > $OUT/pt_$r.json 2> $OUT/pt_$r.err || exit 1
done
