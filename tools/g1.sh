set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for tw in 4096 6144; do
for v in ND L R R2 NW; do
  SPG_TARGET_WAVES=$tw SPG_GPU_LIB=tools/_variants/lib$v.so timeout -k 10 200 python tools/kbench.py --tag ${v}_tw$tw >> gpurun_out/kb.log 2>&1
done; done
cat gpurun_out/kb.log
