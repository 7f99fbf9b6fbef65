#!/bin/bash
# g_tw.sh: target-waves sweep (TWS) of variant(s) VARIANTS at DEPTHS
cd /root/repo
export TMPDIR=/tmp
for d in ${DEPTHS:-10000}; do
for v in ${VARIANTS:-B}; do
for tw in ${TWS:-16384 6144 3072}; do
  SPG_TARGET_WAVES=$tw SPG_GPU_LIB=tools/_variants/lib_$v.so timeout -k 10 300 python tools/kbench.py --tag $v --depth $d --calls-only --iters 40 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tag'], $d, $tw, round(d['acc_ms']*1000,1), round(d['acc_min_ms']*1000,1), round(d['fin_ms']*1000,1))" || exit 1
done; done; done
