#!/bin/bash
# round_check.sh <outdir>: the round-end sequence on one GPU — the -m gpu suite, smoke(), then the default
# bench line (all nested lines, end to end, CPU baselines).  Each step under its own limit; stops at the first failure.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/${1:-gpurun_out/check}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed" | tee -a $OUT/fail.log; exit 1; }
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed" | tee -a $OUT/fail.log; exit 1; }
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed" | tee -a $OUT/fail.log; exit 1; }
