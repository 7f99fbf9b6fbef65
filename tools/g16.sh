#!/bin/bash
# g16.sh: parity of the fast-path variants, then timing A/B
cd /root/repo
export TMPDIR=/tmp
for v in X1 F1; do
  SPG_GPU_LIB=tools/_variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t16_$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(tail -1 gpurun_out/t16_$v.log)"; [ $rc = 0 ] || exit 1
done
VARIANTS="A0 F1n F2n X1n" DEPTHS="10000 1000" bash tools/gab.sh || exit 1
