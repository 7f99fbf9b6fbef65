#!/bin/bash
# r05k: parallel inflater after two-level tables + cooperative dependent matches: tests, bench, instrumented phase split
OUT=gpurun_out/${1:-r05k}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_inflate_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/inflate_tests.log 2>&1 || { tail -40 $OUT/inflate_tests.log; exit 1; }
tail -2 $OUT/inflate_tests.log
timeout -k 10 300 python3 -u tools/inflate_bench.py > $OUT/inflate_bench.json 2> $OUT/inflate_bench.err || { tail -20 $OUT/inflate_bench.err; exit 1; }
cat $OUT/inflate_bench.json
