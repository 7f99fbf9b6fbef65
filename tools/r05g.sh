#!/bin/bash
# r05g: kernel-level evidence of the r05 device pileup path — rocprofv3 kernel stats of the end-to-end leg (lone
# process_bam with the BAM in HBM: k_inflate, k_crc32, k_bam_*, k_fill*, the accumulate kernels), FETCH_SIZE and
# WRITE_SIZE passes (one counter group per run), then the headline bench leg under rocprofv3 (tools/prof_bench.sh)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05g}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/e2e_trace -o run --output-format csv -- \
    python3 $ROOT/tools/e2e_only.py 4 0 16 > $OUT/e2e_trace.log 2>&1 || { echo "e2e trace failed"; tail -20 $OUT/e2e_trace.log; exit 1; }
i=0
for pass in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $pass -d $OUT/e2e_pmc$i -o run --output-format csv -- \
      python3 $ROOT/tools/e2e_only.py 2 0 16 > $OUT/e2e_pmc$i.log 2>&1 || { echo "e2e pmc $pass failed"; tail -20 $OUT/e2e_pmc$i.log; exit 1; }
done
bash $ROOT/tools/prof_bench.sh gpurun_out/${1:-r05g}/main || { echo "prof_bench failed"; exit 1; }
python3 $ROOT/tools/prof_sum.py $OUT > $OUT/summary.txt 2>&1
find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete
find $OUT -name "*.log" -size +1M -delete
cat $OUT/summary.txt
