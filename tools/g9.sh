set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for k in 1 2; do timeout -k 10 300 python tools/kbench.py --tag head --calls-only --iters 40; done
timeout -k 10 300 python tools/kbench.py --tag head1000 --depth 1000 --calls-only --iters 40
