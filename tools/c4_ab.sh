#!/bin/bash
# c4_ab.sh <outdir>: config 4 live form (10,000 per-BAM batches) with the run kernel's LPC from the default rule
# (LPC 2: 32-column units, 4 KiB slots) and forced to 4 (16-column units), interleaved twice.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/${1:-gpurun_out/c4ab}
mkdir -p $OUT
cd /tmp
B="$ROOT/bench.py --no-parity --no-chr1 --no-e2e --no-cpu-baseline --reps 3 --steps 3 --warmup 2"
for r in 1 2; do
  timeout -k 10 200 python3 -u $B > $OUT/lpcdef_$r.log 2>&1 || exit 1
  SPG_RUN_LPC=${ALT_LPC:-4} timeout -k 10 200 python3 -u $B > $OUT/lpc${ALT_LPC:-4}_$r.log 2>&1 || exit 1
done
