# r04g: the round-end sequence (GPU suite, smoke, the driver's default bench line) + the per-BAM probe
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04g}; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
s=$(date +%s)
timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"
timeout -k 10 300 python3 -u tools/per_bam_probe.py 3000 $OUT/probe.jsonl > $OUT/probe.log 2>&1 || { echo "probe failed"; tail -20 $OUT/probe.log; exit 1; }
echo done
