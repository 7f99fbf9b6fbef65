#!/bin/bash
# pmc_inflate_bytes.sh <outdir>: FETCH_SIZE / WRITE_SIZE passes (separate rocprofv3 runs) over tools/inflate_bench.py;
# summary: k_inflate_par and k_crc32 bytes per launch (FETCH_SIZE in KiB, x2 on gfx950 for wide streaming reads)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/${1:-gpurun_out/inflate_bytes}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
i=0
for pass in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass -d $OUT/pmc$i -o run --output-format csv -- python3 $ROOT/tools/inflate_bench.py > $OUT/pmc$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 $ROOT/tools/pmc_report.py $OUT k_inflate_par > $OUT/summary.txt
python3 $ROOT/tools/pmc_report.py $OUT k_crc32 >> $OUT/summary.txt
find $OUT -name "*.csv" -delete
cat $OUT/summary.txt
