#!/bin/bash
# g_ab.sh: GPU parity tests of the in-tree build, then A/B timing of tools/_variants/lib_{VARIANTS}.so
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 1; }
tail -2 gpurun_out/pytest_ab.log
bash tools/gab.sh
