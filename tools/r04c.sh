# r04c: full -m gpu suite, the per-BAM probe and the new bench legs
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04c}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_live_loop_gpu.py -x -q --timeout 240 --timeout-method thread > $OUT/new_tests.log 2>&1 || { echo "new tests failed"; tail -40 $OUT/new_tests.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python3 -u tools/per_bam_probe.py 3000 $OUT/probe.jsonl > $OUT/probe.log 2>&1 || { echo "probe failed"; tail -20 $OUT/probe.log; exit 1; }
timeout -k 10 500 python3 -u bench.py --legs sars1k,config4 --reps 10 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
echo done
