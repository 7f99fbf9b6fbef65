#!/bin/bash
# g12.sh: explicit PF=3 ring / nt loads A/B, target-waves sweep for the winner
cd /root/repo
export TMPDIR=/tmp
VARIANTS="A B C D" DEPTHS="10000 1000" bash tools/gab.sh || exit 1
for tw in 8192 12288 24576; do for v in A B; do
  SPG_TARGET_WAVES=$tw SPG_GPU_LIB=tools/_variants/lib_$v.so timeout -k 10 300 python tools/kbench.py --tag $v-tw$tw --calls-only --iters 40 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tag'], round(d['acc_ms']*1000,1), round(d['acc_min_ms']*1000,1))" || exit 1
done; done
