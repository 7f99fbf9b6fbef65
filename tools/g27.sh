#!/bin/bash
cd /root/repo
export TMPDIR=/tmp
VARIANTS="P2 P3" DEPTHS="10000 1000" bash tools/gab.sh || exit 1
for v in P2 P3; do
  SPG_GPU_LIB=tools/_variants/lib_$v.so timeout -k 10 400 python tools/kbench.py --tag $v --depth 100000 --calls-only --iters 5 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tag'], 100000, round(d['acc_ms']*1000,1), round(d['acc_min_ms']*1000,1))" || exit 1
done
