set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base w4 r4; do
  SPG_GPU_LIB=tools/_variants/lib_$v.so timeout -k 10 300 python tools/kbench.py --tag $v --calls-only --iters 40
done
cd /tmp
timeout -k 10 120 rocprofv3 -L > /root/repo/gpurun_out/counters.txt 2>&1 || true
for pass in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY" "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_BRANCH" ; do
  i=$((i+1))
  SPG_GPU_LIB=/root/repo/tools/_variants/lib_w4.so timeout -k 10 200 rocprofv3 --pmc $pass -d /root/repo/gpurun_out/ic$i -o run --output-format csv -- python /root/repo/tools/kbench.py --calls-only --iters 2 > /root/repo/gpurun_out/ic$i.log 2>&1 || echo "pass $i failed"
done
