# r04zk: same-box interleaved A/B of the deep kernel: current vs SPG_CLIP (chunk loads clipped at their column's end,
# _lib/ab/clip.so); main + parity mode, 3 rounds; then FETCH_SIZE per launch of each (kbench, calls-only)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04zk}; mkdir -p $OUT
L=$GRAFT_REPO_ROOT/covid-spings-variant-caller_amd/_lib
B="bench.py --legs parity --no-cpu-baseline --reps 10"
for r in 1 2 3; do
  for v in cur clip; do
    if [ $v = cur ]; then lib=$L/libspings_gpu.so; else lib=$L/ab/$v.so; fi
    SPG_GPU_LIB=$lib timeout -k 10 200 python3 -u $B > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { echo "$v failed"; tail -5 $OUT/${v}_$r.err; exit 1; }
    python3 - $OUT/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "main", round(d["ms_per_step"] * 1e3, 1), round(d["roofline"]["kernel_ms"] * 1e3, 1), "parity", round(d["parity_mode"]["ms_per_step"] * 1e3, 1), round(d["parity_mode"]["roofline"]["kernel_ms"] * 1e3, 1))
PY
  done
done
cd /tmp
for v in cur clip; do
  if [ $v = cur ]; then lib=$L/libspings_gpu.so; else lib=$L/ab/$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    SPG_GPU_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $c -d $GRAFT_REPO_ROOT/$OUT/pmc_${v}_$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --calls-only --iters 3 > $GRAFT_REPO_ROOT/$OUT/pmc_${v}_$c.log 2>&1 || { echo "pmc $v $c failed"; exit 1; }
  done
done
python3 $GRAFT_REPO_ROOT/tools/pmc_sum.py $GRAFT_REPO_ROOT/$OUT "k_acc_seg<4" > $GRAFT_REPO_ROOT/$OUT/pmc_sum.txt 2>&1; cat $GRAFT_REPO_ROOT/$OUT/pmc_sum.txt
