set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/kb.log
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for tw in 16384 8192; do
for v in BASE T4 T0; do
  SPG_TARGET_WAVES=$tw SPG_GPU_LIB=tools/_variants/lib$v.so timeout -k 10 200 python tools/kbench.py --tag ${v}_tw$tw 2>/dev/null >> gpurun_out/kb.log
done; done
cut -c1-130 gpurun_out/kb.log
SPG_GPU_LIB=tools/_variants/libT4.so timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM -d gpurun_out/abl2/T4 -o run --output-format csv -- python3 tools/kbench.py --iters 2 > gpurun_out/abl2/T4.log 2>&1
