#!/bin/bash
# g22.sh: GPU tests (incl. offsets past 2^31), then the 100,000x kbench batch that faulted before the fix
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest22.log 2>&1 || { tail -30 gpurun_out/pytest22.log; exit 1; }
tail -2 gpurun_out/pytest22.log
timeout -k 10 600 python -u tools/kbench.py --tag fix --depth 100000 --calls-only --iters 5 || exit 1
timeout -k 10 300 python -u tools/kbench.py --tag fix --depth 10000 --calls-only --iters 30 || exit 1
