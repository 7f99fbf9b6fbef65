#!/bin/bash
cd /root/repo
export TMPDIR=/tmp
VARIANTS="B0 N4 N5" DEPTHS="10000 1000" bash tools/gab.sh || exit 1
for tw in 8192 32768; do
  SPG_TARGET_WAVES=$tw SPG_GPU_LIB=tools/_variants/lib_B0.so timeout -k 10 300 python tools/kbench.py --tag B0-tw$tw --calls-only --iters 40 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tag'], round(d['acc_ms']*1000,1), round(d['acc_min_ms']*1000,1))" || exit 1
done
