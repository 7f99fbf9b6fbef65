#!/bin/bash
# deep_ab.sh <outdir>: the sars10k metric point, interleaved A/B of deep-kernel variants (two rounds):
#   base  — the default build (G = 3 under the fused finalize's 4-record ring)
#   nb8   — _lib/ab/libspings_gpu_nb8.so (-DSPG_NB=8) with G = 8: one wave generation (3,738 waves)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/${1:-gpurun_out/deepab}
mkdir -p $OUT
cd /tmp
B="$ROOT/bench.py --no-parity --many-batches 0 --no-chr1 --runs-batches 0 --no-e2e --no-cpu-baseline --reps 10"
for r in 1 2; do
  timeout -k 10 120 python3 -u $B > $OUT/base_$r.log 2>&1 || exit 1
  SPG_GPU_LIB=$ROOT/covid-spings-variant-caller_amd/_lib/ab/libspings_gpu_nb8.so SPG_TARGET_WAVES=4096 SPG_TAIL_WAVES=0 \
    timeout -k 10 120 python3 -u $B > $OUT/nb8_$r.log 2>&1 || exit 1
  SPG_GPU_LIB=$ROOT/covid-spings-variant-caller_amd/_lib/ab/libspings_gpu_nb8.so SPG_TARGET_WAVES=5000 SPG_TAIL_WAVES=0 \
    timeout -k 10 120 python3 -u $B > $OUT/nb8g6_$r.log 2>&1 || exit 1
done
