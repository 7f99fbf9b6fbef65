#!/bin/bash
# r05o: end-to-end leg with k_inflate_par (lone process_bam with the BAM in HBM, process_bams, VCQueue loop), then the
# e2e path's kernels under rocprofv3 --kernel-trace --stats
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05o}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
SPP_TIMING=1 timeout -k 10 600 python3 -u bench.py --no-main --legs e2e --e2e-many 16 > $OUT/e2e.json 2> $OUT/e2e.err || { tail -40 $OUT/e2e.err; exit 1; }
python3 - $OUT/e2e.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["end_to_end"]
for tag in ("parity_mode_max_depth_8000", "uncapped"):
    e = d[tag]
    print(tag, "device %.3g" % e["positions_per_s_per_bam"], "records %.3g" % e["records_plan_path"]["positions_per_s_per_bam"],
          "process_bams %.3g" % e["process_bams"]["positions_per_s_per_bam"])
    print("  breakdown", {k: round(v, 2) if isinstance(v, float) else v for k, v in e["breakdown_one_bam_device"].items()})
    v = e["vcqueue_loop"]
    print("  vcqueue", {k: v[k] for k in ("ms_per_bam", "process_bam_ms", "create_checkpoint_ms", "write_vcf_ms")})
PY
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/e2e_trace -o run --output-format csv -- \
    python3 $ROOT/tools/e2e_only.py 4 0 16 > $OUT/e2e_trace.log 2>&1 || { echo "e2e trace failed"; tail -20 $OUT/e2e_trace.log; exit 1; }
python3 $ROOT/tools/prof_sum.py $OUT > $OUT/summary.txt 2>&1
find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete
head -16 $OUT/summary.txt
