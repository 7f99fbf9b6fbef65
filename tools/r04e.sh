# r04e: deep-kernel dynamic-tail A/B (interleaved), main point + parity mode; then sars1k with and without
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04e}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_live_loop_gpu.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $OUT/t.log 2>&1 || { echo "tests failed"; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for r in 1 2; do
  for cfg in "0 0" "0.15 0" "0.15 1" "0.3 0"; do
    set -- $cfg
    SPG_DYN_FRAC=$1 SPG_DYN_HALF=$2 timeout -k 10 200 python3 -u bench.py --legs parity --reps 10 > $OUT/ab_$1_$2_$r.json 2> $OUT/ab_$1_$2_$r.err || { echo "bench $cfg failed"; tail -20 $OUT/ab_$1_$2_$r.err; exit 1; }
  done
done
for f in 0 0.15; do
  SPG_DYN_FRAC=$f timeout -k 10 200 python3 -u bench.py --legs sars1k --reps 5 > $OUT/s1k_$f.json 2> $OUT/s1k_$f.err || { echo "sars1k failed"; exit 1; }
done
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/ab_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["roofline"]["kernel_ms"] * 1e3, 2), "us", round(d["roofline"]["frac"], 4),
          "parity", round(d["parity_mode"]["roofline"]["kernel_ms"] * 1e3, 2), round(d["parity_mode"]["roofline"]["frac"], 4))
for f in sorted(glob.glob(sys.argv[1] + "/s1k_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])["sars1k"]
    print(f.split("/")[-1], d["ms_per_step"], round(d["roofline"]["frac"], 4), d["roofline"]["kernel_ms"], d["finalize_ms"])
PY
echo done
