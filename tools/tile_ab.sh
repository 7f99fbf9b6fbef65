#!/bin/bash
# tile_ab.sh <outdir> [bench args...]: chr1 30x through k_acc_tile — grid-size A/B, then SQ counter passes for the
# tile kernel and the r02 kernel (SPG_SHALLOW=old).  Counters only in the --pmc passes (no tracing domains).
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/${1:-gpurun_out/tileab}
shift || true
EXTRA="$*"
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
B="$ROOT/bench.py --workload chr1_30x --no-cpu-baseline --no-e2e --no-parity --reps 3 --steps 3 --warmup 2 $EXTRA"
for nb in ${TILE_BLOCKS_LIST:-1280 1024}; do
  SPG_TILE_BLOCKS=$nb timeout -k 10 200 python3 -u $B > $OUT/nb$nb.log 2>&1 || { echo "nb$nb failed" >> $OUT/fail.log; exit 1; }
done
P="$ROOT/bench.py --workload chr1_30x --no-cpu-baseline --no-e2e --no-parity --reps 1 --steps 2 --warmup 1 --min-ms 1 $EXTRA"
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
            "FETCH_SIZE"; do
  i=$((i+1))
  for mode in new old; do
    if [ $mode = old ]; then export SPG_SHALLOW=old; else unset SPG_SHALLOW; fi
    timeout -s KILL 200 rocprofv3 --pmc $pass -d $OUT/p${i}_$mode -o run --output-format csv -- python3 -u $P > $OUT/p${i}_$mode.log 2>&1 || { echo "pass $i $mode failed" >> $OUT/fail.log; exit 1; }
  done
done
unset SPG_SHALLOW
