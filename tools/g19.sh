#!/bin/bash
# g19.sh: GPU tests of the in-tree build, then kernel timings at 1,000x / 10,000x / 100,000x
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest19.log 2>&1 || { tail -40 gpurun_out/pytest19.log; exit 1; }
tail -2 gpurun_out/pytest19.log
for d in 1000 10000 100000; do
  timeout -k 10 300 python tools/kbench.py --tag cur --depth $d --calls-only --iters 20 || exit 1
done
