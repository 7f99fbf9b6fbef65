# r04t: deep kernel with soffset chunk loads + lane-held column descriptors: GPU suite, main/parity/sars100k lines, rocprof of main
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04t}; mkdir -p $OUT
[ -n "$SKIPT" ] || { timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --legs sars100k,sars100k_capped > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("main", round(d["ms_per_step"] * 1e3, 1), round(d["roofline"]["kernel_ms"] * 1e3, 1), round(d["roofline"]["frac"], 3))
p = d["parity_mode"]; print("parity", round(p["ms_per_step"] * 1e3, 1), round(p["roofline"]["kernel_ms"] * 1e3, 1), round(p["roofline"]["frac"], 3))
s = d["sars100k"]; print("s100k", round(s["ms_per_step"] * 1e3, 1), round(s["roofline"]["frac"], 3), round(s["parity_mode"]["ms_per_step"] * 1e3, 1), round(s["parity_mode"]["roofline"]["frac"], 3))
PY
bash tools/prof_legs.sh $OUT/prof main > $OUT/prof.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof.log; exit 1; }
head -3 $OUT/prof/main/trace/run_kernel_stats.csv | cut -c1-160
