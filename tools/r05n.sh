#!/bin/bash
# r05n: k_inflate_par ring size / waves-per-SIMD A/B (tools/build_ab.sh variants), interleaved, kernel ms per 10,000x BAM
OUT=gpurun_out/r05n
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in default r4k r4k_w4 r8k_w4; do
    if [ $v = default ]; then cmd="tools/inflate_bench.py"; else cmd="tools/ab_run.py $v.so tools/inflate_bench.py"; fi
    timeout -k 10 200 python3 -u $cmd > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { echo "$v failed"; tail -5 $OUT/${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${v}_$rep.json')); print('$v', [r['kernel_ms'] for r in d['runs']], 'identical', d['identical'], 'lane', [r['lane_kernel_members'] for r in d['runs']][-1])"
  done
done
