#!/bin/bash
# pmc.sh <outdir> : rocprofv3 PMC passes (counters only, kernel-trace allowed) over tools/kbench.py
set -e
OUT=${1:-gpurun_out/pmc}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/$OUT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 python $ROOT/tools/kbench.py --calls-only --iters 2 > /dev/null 2>&1   # warm the data cache
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_IFETCH GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $pass -d $ROOT/$OUT/p$i -o run --output-format csv -- python $ROOT/tools/kbench.py --calls-only --iters 2 > $ROOT/$OUT/p$i.log 2>&1 || echo "pass $i failed" >> $ROOT/$OUT/fail.log
done
