#!/bin/bash
# r05zr: GPU busy time inside the lone process_bam stream and process_bams (kernel + memory-copy trace)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zr}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/trace -o run --output-format csv -- python3 $ROOT/tools/pbams_trace.py 6 16 $OUT/marks.json > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; find $OUT -name "*.csv" -delete; exit 1; }
SPP_TIMING=1 timeout -k 10 300 python3 $ROOT/tools/pbams_trace.py 6 16 > $OUT/timing.log 2>&1 || { tail -20 $OUT/timing.log; find $OUT -name "*.csv" -delete; exit 1; }
python3 $ROOT/tools/pbams_gaps.py $OUT/trace $OUT/marks.json > $OUT/gaps.txt 2>&1
find $OUT -name "*.csv" -delete
cat $OUT/gaps.txt; grep "plan_fields" $OUT/timing.log | tail -8; tail -1 $OUT/timing.log
