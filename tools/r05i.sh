#!/bin/bash
# r05i: the parallel inflater (k_inflate_par) on the GPU: inflate tests, the 10,000x BAM inflate bench (kernel ms, members
# left to the lane kernel, identical to gzip), then the device-pileup / live-caller GPU tests that inflate BAMs in HBM
OUT=gpurun_out/r05i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_inflate_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/inflate_tests.log 2>&1 || { tail -40 $OUT/inflate_tests.log; exit 1; }
tail -3 $OUT/inflate_tests.log
timeout -k 10 300 python3 -u tools/inflate_bench.py > $OUT/inflate_bench.json 2> $OUT/inflate_bench.err || { tail -20 $OUT/inflate_bench.err; exit 1; }
cat $OUT/inflate_bench.json
timeout -k 10 600 python3 -u -m pytest tests/test_device_pileup_gpu.py tests/test_live_caller_gpu.py -x -q --timeout 240 --timeout-method thread > $OUT/pileup_tests.log 2>&1 || { tail -40 $OUT/pileup_tests.log; exit 1; }
tail -3 $OUT/pileup_tests.log
