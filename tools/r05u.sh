#!/bin/bash
# r05u: device-fill tests, kernel trace of the e2e leg, FETCH / WRITE of the fill kernels
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05u}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_inflate_gpu.py tests/test_device_pileup_gpu.py tests/test_live_caller_gpu.py -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 -u tools/inflate_bench.py > $OUT/inflate_bench.json 2> $OUT/inflate_bench.err || { tail -20 $OUT/inflate_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/inflate_bench.json')); print('inflate', [r['kernel_ms'] for r in d['runs']], d['identical'], d['runs'][-1]['lane_kernel_members'])"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $ROOT/tools/e2e_only.py 2 0 16 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
i=0
for pass in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass -d $OUT/pmc$i -o run --output-format csv -- \
      python3 $ROOT/tools/e2e_only.py 2 0 16 > $OUT/pmc$i.log 2>&1 || { echo "pmc $pass failed"; tail -20 $OUT/pmc$i.log; exit 1; }
done
python3 $ROOT/tools/prof_sum.py $OUT > $OUT/summary.txt 2>&1
find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete
find $OUT -name "*.log" -size +1M -delete
grep -i "f2_\|inflate\|crc\|bam_" $OUT/summary.txt | head -30
