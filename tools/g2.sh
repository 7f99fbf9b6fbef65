set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
rm -f gpurun_out/kb.log
for tw in 16384 8192; do
for v in M4 C4; do
  SPG_TARGET_WAVES=$tw SPG_GPU_LIB=tools/_variants/lib$v.so timeout -k 10 200 python tools/kbench.py --iters 40 --tag ${v}_tw$tw 2>/dev/null >> gpurun_out/kb.log
done; done
cut -c1-110 gpurun_out/kb.log
