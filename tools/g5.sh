cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 7 4; do
  SPG_RING=$r timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_live_caller_gpu.py -m gpu -q > gpurun_out/pytest_ring$r.log 2>&1
  echo "ring $r rc=$?"; tail -3 gpurun_out/pytest_ring$r.log
done
for r in 0 7 4; do
  SPG_RING=$r timeout -k 10 300 python tools/kbench.py --tag ring$r --calls-only --iters 40 || exit 1
done
