# gab.sh: alternate A/B kernel variants on one box (VARIANTS, DEPTHS)
cd /root/repo
export TMPDIR=/tmp
for rep in 1 2; do
for d in ${DEPTHS:-10000 1000}; do
for v in ${VARIANTS:-A C}; do
  SPG_GPU_LIB=tools/_variants/lib_$v.so timeout -k 10 300 python tools/kbench.py --tag $v --depth $d --calls-only --iters 40 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tag'], $d, round(d['acc_ms']*1000,1), round(d['acc_min_ms']*1000,1), round(d['fin_ms']*1000,1))" || exit 1
done; done; done
