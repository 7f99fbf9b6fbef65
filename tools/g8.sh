cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/kbench.py --tag head --calls-only --iters 40 || exit 1
for v in ${VARIANTS:-e1 e5 e6 e7 e8}; do
  SPG_GPU_LIB=tools/_variants/lib_$v.so timeout -k 10 300 python tools/kbench.py --tag $v --calls-only --iters 40 || exit 1
done
