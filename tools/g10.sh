cd /root/repo
export TMPDIR=/tmp
for tw in 16384 8192 4096 2048; do
  SPG_TARGET_WAVES=$tw timeout -k 10 300 python tools/kbench.py --tag tw$tw --depth 1000 --calls-only --iters 40 || exit 1
  SPG_TARGET_WAVES=$tw timeout -k 10 300 python tools/kbench.py --tag tw$tw --calls-only --iters 40 || exit 1
done
