#!/bin/bash
# r05s: FETCH_SIZE / WRITE_SIZE of the new inflater and the e2e device-path kernels (one counter group per pass), and the
# inflater's SQ counters (tools/pmc_inflate.sh)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/r05s
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
i=0
for pass in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass -d $OUT/e2e_pmc$i -o run --output-format csv -- \
      python3 $ROOT/tools/e2e_only.py 2 0 16 > $OUT/e2e_pmc$i.log 2>&1 || { echo "e2e pmc $pass failed"; tail -20 $OUT/e2e_pmc$i.log; exit 1; }
done
python3 $ROOT/tools/prof_sum.py $OUT > $OUT/summary.txt 2>&1
bash $ROOT/tools/pmc_inflate.sh gpurun_out/r05s/sq > /dev/null || { echo "sq pmc failed"; exit 1; }
find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete
find $OUT -name "*.log" -size +1M -delete
cat $OUT/summary.txt; head -20 $OUT/sq/summary.txt
