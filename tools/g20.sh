#!/bin/bash
# g20.sh: GPU tests of the in-tree build, then kernel timings at 1,000x / 10,000x
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest20.log 2>&1 || { tail -40 gpurun_out/pytest20.log; exit 1; }
tail -2 gpurun_out/pytest20.log
for rep in 1 2; do for d in 1000 10000; do
  timeout -k 10 300 python tools/kbench.py --tag cur --depth $d --calls-only --iters 30 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($d, round(d['acc_ms']*1000,1), round(d['acc_min_ms']*1000,1), round(d['fin_ms']*1000,1), round(d['step_ms']*1000,1), d['n_cand'])" || exit 1
done; done
