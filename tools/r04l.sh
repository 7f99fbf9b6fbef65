# r04l: k_count_cols A/B (LPC, workgroups per CU) on sars1k; the count path forced on the 10,000x headline and 100,000x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04l}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "mid_depth" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {  # name env... -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --reps 5 --no-cpu-baseline $BARGS > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; exit 1; }
  python3 - $OUT/$name.json $name $LEG <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d[sys.argv[3]] if sys.argv[3] != "main" else d
print(sys.argv[2], round(s["ms_per_step"], 4), round(s["roofline"]["kernel_ms"], 4), round(s["roofline"]["frac"], 3))
PY
}
BARGS="--no-main --legs sars1k"; LEG=sars1k
for l in 8 16 32; do run s1k_l$l SPG_COUNT_LPC=$l; done
for b in 512 1024 2048; do run s1k_b$b SPG_COUNT_BLOCKS=$b; done
BARGS="--legs none --no-parity"; LEG=main
run s10k_fused SPG_COUNT_COLS=-1
for l in 32 64; do run s10k_count_l$l SPG_COUNT_COLS=1 SPG_COUNT_LPC=$l; done
BARGS="--no-main --legs sars100k"; LEG=sars100k
run s100k_fused SPG_COUNT_COLS=-1
run s100k_count SPG_COUNT_COLS=1 SPG_COUNT_LPC=64
