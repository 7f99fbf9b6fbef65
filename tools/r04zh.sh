# r04zh: where a records plan's time goes with the GPU inflater (SPP_TIMING), end-to-end leg forced to GPU inflate
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04zh}; mkdir -p $OUT
SPG_GPU_INFLATE=1 SPP_TIMING=1 timeout -k 10 300 python3 -u tools/e2e_only.py 4 0 16 > $OUT/e2e_gpu.json 2> $OUT/e2e_gpu.err || { echo "e2e failed"; tail -20 $OUT/e2e_gpu.err; exit 1; }
grep -A1 "gpu inflate" $OUT/e2e_gpu.err | tail -24
