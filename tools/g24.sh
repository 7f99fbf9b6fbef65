#!/bin/bash
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest24.log 2>&1 || { tail -30 gpurun_out/pytest24.log; exit 1; }
tail -1 gpurun_out/pytest24.log
for d in 1000 10000 1000 10000; do
  timeout -k 10 300 python tools/kbench.py --tag G --depth $d --calls-only --iters 30 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($d, round(d['acc_ms']*1000,1), round(d['acc_min_ms']*1000,1), round(d['fin_ms']*1000,1), round(d['step_ms']*1000,1))" || exit 1
done
