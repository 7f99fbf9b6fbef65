#!/bin/bash
# r05zg: SQ counters of the e2e device-path kernels (k_f2_fill's LDS form): two passes over tools/e2e_only.py
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zg}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_BRANCH"
i=0
for pass in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass -d $OUT/pmc$i -o run --output-format csv -- \
      python3 $ROOT/tools/e2e_only.py 2 0 16 > $OUT/pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 $ROOT/tools/pmc_report.py $OUT k_f2_fill > $OUT/summary.txt
python3 $ROOT/tools/pmc_report.py $OUT k_bam_ >> $OUT/summary.txt
find $OUT -name "*.csv" -delete
find $OUT -name "*.log" -size +1M -delete
cat $OUT/summary.txt
