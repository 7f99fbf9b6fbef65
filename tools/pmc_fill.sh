#!/bin/bash
# pmc_fill.sh <outdir> [max_depth]: kernel trace + SQ counter passes (one rocprofv3 run each) over tools/fill_bench.py
# (open + GPU plan + fill of the 10,000x BAM); summary: tools/pmc_report.py <outdir> k_f2_fill
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/$1
MD=${2:-0}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- \
    python3 $ROOT/tools/fill_bench.py 10000 $MD 6 > $OUT/kt.log 2>&1 || { echo "trace failed"; tail -5 $OUT/kt.log; exit 1; }
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_BRANCH"
i=0
for pass in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass -d $OUT/pmc$i -o run --output-format csv -- \
      python3 $ROOT/tools/fill_bench.py 10000 $MD 3 > $OUT/pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 $ROOT/tools/pmc_report.py $OUT k_f2_fill > $OUT/summary.txt
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT -name "*.csv" ! -name kernel_stats.csv -delete
cat $OUT/summary.txt
