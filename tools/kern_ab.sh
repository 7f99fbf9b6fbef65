#!/bin/bash
# kern_ab.sh <outdir> [bench args...]: chr1 30x through each shallow-kernel form in $MODES (lite = k_acc_lite, the
# default; tile = k_acc_tile, SPG_LITE=0; old = the r02 k_acc_one, SPG_SHALLOW=old), then a kernel-trace summary and
# the counter passes for each.  Counters only in the --pmc passes (no tracing domains).
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/${1:-gpurun_out/kernab}
shift || true
EXTRA="$*"
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
setmode() {
  unset SPG_SHALLOW SPG_LITE
  case $1 in
    tile) export SPG_LITE=0 ;;
    old) export SPG_SHALLOW=old ;;
  esac
}
B="$ROOT/bench.py --workload chr1_30x --no-cpu-baseline --no-e2e --no-parity --reps 3 --steps 3 --warmup 2 $EXTRA"
for mode in ${MODES:-lite tile old}; do
  setmode $mode
  timeout -k 10 200 python3 -u $B > $OUT/bench_$mode.log 2>&1 || { echo "bench $mode failed" >> $OUT/fail.log; exit 1; }
done
P="$ROOT/bench.py --workload chr1_30x --no-cpu-baseline --no-e2e --no-parity --reps 1 --steps 2 --warmup 1 --min-ms 1 $EXTRA"
for mode in ${PMC_MODES:-lite}; do
  setmode $mode
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $OUT/kt_$mode -o run --output-format csv -- python3 -u $P > $OUT/kt_$mode.log 2>&1 || { echo "kt $mode failed" >> $OUT/fail.log; exit 1; }
  i=0
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" \
              "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
              "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $pass -d $OUT/p${i}_$mode -o run --output-format csv -- python3 -u $P > $OUT/p${i}_$mode.log 2>&1 || { echo "pass $i $mode failed" >> $OUT/fail.log; exit 1; }
  done
done
setmode lite
