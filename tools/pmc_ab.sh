#!/bin/bash
# pmc_ab.sh <outdir> <variants...>: instruction-mix PMC passes of tools/kbench.py per variant library
OUT=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/$OUT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 python $ROOT/tools/kbench.py --calls-only --iters 2 > /dev/null 2>&1   # warm the data cache
for v in "$@"; do
  i=0
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
              "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
              "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_IFETCH GRBM_COUNT"; do
    i=$((i+1))
    SPG_GPU_LIB=$ROOT/tools/_variants/lib_$v.so timeout -k 10 120 rocprofv3 --pmc $pass -d $ROOT/$OUT/$v/p$i -o run --output-format csv -- python $ROOT/tools/kbench.py --calls-only --iters 2 > $ROOT/$OUT/$v.p$i.log 2>&1 || { echo "pass $v $i failed"; exit 1; }
  done
done
