set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for v in ${VARIANTS:-base w4 w5 w6}; do
  for co in --calls-only ""; do
    SPG_GPU_LIB=tools/_variants/lib_$v.so timeout -k 10 300 python tools/kbench.py --tag $v $co --iters 40
  done
done
