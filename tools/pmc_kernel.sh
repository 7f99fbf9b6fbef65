#!/bin/bash
# pmc_kernel.sh <outdir> <bench args...>: SQ / TA / TCP counter passes (one rocprofv3 --pmc run each,
# within the per-block limits) over a bench.py workload; summarize with tools/pmc_report.py.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/$1
shift
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_BRANCH TA_TA_BUSY_sum TA_BUFFER_COALESCED_READ_CYCLES_sum"
P3="TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"
i=0
for pass in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass -d $OUT/pmc$i -o run --output-format csv -- \
      python3 $ROOT/bench.py "$@" > $OUT/pmc$i.log 2>&1
done
