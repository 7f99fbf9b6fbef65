#!/bin/bash
# r05zo: round check of the final r05 tree — the -m gpu suite, smoke(), the default bench line; then the headline's
# rocprofv3 kernel trace + FETCH/WRITE passes (tools/prof_bench.sh), and the end-to-end leg's kernel trace + FETCH/WRITE
# of the BAM-path kernels (k_f2_fill's write traffic).  Each step under its own limit; stops at the first failure.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
N=${1:-r05zo}
OUT=$ROOT/gpurun_out/$N
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
if [ -z "$NO_CHECK" ]; then
  bash tools/round_check.sh gpurun_out/$N/check || exit 1
  tail -1 $OUT/check/gpu_tests.log; tail -2 $OUT/check/smoke.log
else
  mkdir -p $OUT/check
  timeout -k 10 600 python3 -u bench.py > $OUT/check/bench.json 2> $OUT/check/bench.err || { echo "bench failed"; tail -5 $OUT/check/bench.err; exit 1; }
fi
bash tools/prof_bench.sh gpurun_out/$N/prof || { echo "prof_bench failed"; find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete; exit 1; }
python3 $ROOT/tools/prof_sum.py $OUT/prof > $OUT/prof/summary.txt 2>&1
find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete
mkdir -p $OUT/e2e
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/e2e/trace -o run --output-format csv -- python3 $ROOT/tools/e2e_only.py 2 0 16 > $OUT/e2e/trace.log 2>&1 || { echo "e2e trace failed"; tail -20 $OUT/e2e/trace.log; find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete; exit 1; }
i=0
for pass in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass -d $OUT/e2e/pmc$i -o run --output-format csv -- \
      python3 $ROOT/tools/e2e_only.py 2 0 16 > $OUT/e2e/pmc$i.log 2>&1 || { echo "pmc $pass failed"; tail -20 $OUT/e2e/pmc$i.log; find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete; exit 1; }
done
python3 $ROOT/tools/prof_sum.py $OUT/e2e > $OUT/e2e/summary.txt 2>&1
find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete
find $OUT -name "*.log" -size +1M -delete
head -14 $OUT/prof/summary.txt
grep -i "f2_\|inflate\|crc\|bam_\|acc_seg" $OUT/e2e/summary.txt | head -30
