# r04zf: end-to-end stream (4 x 10,000x BAMs, 16 threads) with the host inflate and with the GPU inflater, same box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04zf}; mkdir -p $OUT
for v in host gpu; do
  if [ $v = gpu ]; then export SPG_GPU_INFLATE=1; else unset SPG_GPU_INFLATE; fi
  SPP_TIMING=1 timeout -k 10 300 python3 -u tools/e2e_only.py 4 0 16 > $OUT/e2e_$v.json 2> $OUT/e2e_$v.err || { echo "e2e $v failed"; tail -20 $OUT/e2e_$v.err; exit 1; }
  python3 - $OUT/e2e_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
for k in ("uncapped", "parity_mode_max_depth_8000"):
    e = d[k]; print(sys.argv[2], k, round(e["positions_per_s_per_bam"]), "process_bams", round(e["process_bams"]["positions_per_s_per_bam"]),
                    "plan ms", round(e["breakdown_one_bam"]["host_plan_records_s"] * 1e3, 1), "gpu ms", round(e["breakdown_one_bam"]["h2d_records_plus_gpu_s"] * 1e3, 1))
PY
done
