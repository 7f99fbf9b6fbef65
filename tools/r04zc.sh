# r04zc: LDS-table GPU inflater: tests, kernel time at 4/8/16 members per block, then the deep kernel's per-XCD ends
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04zc}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_inflate_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
for m in 4 2 8; do
  SPG_INFLATE_MPW=$m timeout -k 10 200 python3 -u tools/inflate_bench.py > $OUT/inflate_$m.json 2> $OUT/inflate_$m.err || { echo "bench $m failed"; tail -10 $OUT/inflate_$m.err; exit 1; }
  echo "mpw $m"; cat $OUT/inflate_$m.json
done
