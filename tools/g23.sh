#!/bin/bash
# g23.sh: columns-per-wave sweep of the current deep kernel (single-generation grids included)
cd /root/repo
export TMPDIR=/tmp
for tw in 16384 4096 3800 2048; do for d in 10000 1000; do
  SPG_TARGET_WAVES=$tw timeout -k 10 300 python tools/kbench.py --tag tw$tw --depth $d --calls-only --iters 30 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tag'], $d, round(d['acc_ms']*1000,1), round(d['acc_min_ms']*1000,1))" || exit 1
done; done
