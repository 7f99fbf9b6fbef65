# r04x: GPU BGZF inflate — tests, the 10,000x BAM's kernel time, the end-to-end stream with it (16 threads); then the
# deep-kernel same-box A/B (r04w)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04x}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_inflate_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "inflate tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for mpw in 16 64 4; do
  SPG_INFLATE_MPW=$mpw timeout -k 10 300 python3 -u tools/inflate_bench.py > $OUT/inflate_$mpw.json 2> $OUT/inflate_$mpw.err || { echo "inflate bench failed"; tail -20 $OUT/inflate_$mpw.err; exit 1; }
  echo "mpw $mpw"; cat $OUT/inflate_$mpw.json
done
SPG_GPU_INFLATE=1 SPP_TIMING=1 timeout -k 10 300 python3 -u tools/e2e_only.py 4 0 16 > $OUT/e2e_gpuinf.json 2> $OUT/e2e_gpuinf.err || { echo "e2e failed"; tail -20 $OUT/e2e_gpuinf.err; exit 1; }
python3 - $OUT/e2e_gpuinf.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
for k in ("uncapped", "parity_mode_max_depth_8000"):
    e = d[k]; print(k, round(e["positions_per_s_per_bam"]), "process_bams", round(e["process_bams"]["positions_per_s_per_bam"]),
                    "plan ms", round(e["breakdown_one_bam"]["host_plan_records_s"] * 1e3, 1), "gpu ms", round(e["breakdown_one_bam"]["h2d_records_plus_gpu_s"] * 1e3, 1))
PY
grep "read_bam_raw" $OUT/e2e_gpuinf.err | tail -2

