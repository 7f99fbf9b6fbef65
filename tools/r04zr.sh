# r04zr: kernel-level evidence of the device pileup path on the final r04 tree: rocprofv3 kernel stats of the
# end-to-end leg (tools/e2e_only.py: 10,000x BAMs through process_bam and process_bams, GPU inflate on by default) —
# k_inflate, k_tile_first, k_pileup_fill, the accumulate kernels — then FETCH_SIZE / WRITE_SIZE passes (counters only,
# one per run); then the headline bench leg under rocprofv3 (tools/prof_bench.sh)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r04zr}
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
bash $ROOT/tools/prof_bench.sh gpurun_out/${1:-r04zr}/main || { echo "prof_bench failed"; exit 1; }

python3 $ROOT/tools/prof_sum.py $OUT > $OUT/summary.txt 2>&1
# keep the summaries only (the traces exceed what gpurun copies back)
find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete
find $OUT -name "*.log" -size +1M -delete
cat $OUT/summary.txt
