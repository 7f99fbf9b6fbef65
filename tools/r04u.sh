# r04u: end-to-end at the box's 16-CPU share: process_bam stream and process_bams (two plans overlapped), phase timings
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04u}; mkdir -p $OUT
SPP_TIMING=1 timeout -k 10 300 python3 -u tools/e2e_only.py 4 0 16 > $OUT/e2e_16.json 2> $OUT/e2e_16.err || { echo "e2e failed"; tail -20 $OUT/e2e_16.err; exit 1; }
python3 - $OUT/e2e_16.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
for k in ("uncapped", "parity_mode_max_depth_8000"):
    e = d[k]; print(k, round(e["positions_per_s_per_bam"]), "process_bams", round(e["process_bams"]["positions_per_s_per_bam"]),
                    "plan ms", round(e["breakdown_one_bam"]["host_plan_records_s"] * 1e3, 1), "gpu ms", round(e["breakdown_one_bam"]["h2d_records_plus_gpu_s"] * 1e3, 1))
PY
grep "read_bam_raw\|simulate" $OUT/e2e_16.err | tail -6
