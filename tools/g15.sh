#!/bin/bash
# g15.sh: parity of kernel variants (GPU parity tests against each variant library)
cd /root/repo
export TMPDIR=/tmp
for v in X1 X2 X3 F1; do
  SPG_GPU_LIB=tools/_variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t15_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/t15_$v.log)"
done
