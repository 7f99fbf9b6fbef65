# r04d: GPU suite, then the deep kernel with / without the XCD-balanced dynamic tail (interleaved A/B), its wave
# timeline, and a rocprof kernel-trace summary of the default bench main point.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04d}; mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
fi
for r in 1 2; do
  for f in 0.25 0; do
    SPG_DYN_FRAC=$f timeout -k 10 200 python3 -u bench.py --legs parity --reps 10 > $OUT/ab_${f}_$r.json 2> $OUT/ab_${f}_$r.err || { echo "bench $f failed"; tail -20 $OUT/ab_${f}_$r.err; exit 1; }
  done
done
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/ab_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["roofline"]["kernel_ms"] * 1e3, 2), "us", round(d["roofline"]["frac"], 4),
          "parity", round(d["parity_mode"]["roofline"]["kernel_ms"] * 1e3, 2), round(d["parity_mode"]["roofline"]["frac"], 4))
PY
timeout -k 10 200 python3 -u tools/wavetimes.py 10000 $OUT/wavetimes.json > $OUT/wavetimes.log 2>&1 || { echo "wavetimes failed"; tail -20 $OUT/wavetimes.log; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/wavetimes.json')); print({k: d[k] for k in ('span_us','per_xcc_span_us','waves','waves_launched')})"
echo done
