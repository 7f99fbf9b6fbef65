cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04a; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_live_loop_gpu.py -x -v --timeout 240 --timeout-method thread > $OUT/new_tests.log 2>&1 || { echo "new tests failed"; tail -30 $OUT/new_tests.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 500 python3 -u bench.py --legs sars1k,sars100k,config4 --reps 10 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
echo done
