#!/bin/bash
# r05h: inflate A/B — where k_inflate's time goes: decode alone (no output), one byte store per symbol (no match
# reads), members per wave 1/2/3/8
set -o pipefail
OUT=gpurun_out/r05h
mkdir -p $OUT
for v in default decode_only decode_only1 decode_only8 token_stores mpw2 default; do
  if [ $v = default ]; then timeout -k 10 200 python -u tools/inflate_bench.py > $OUT/inflate_$v.json 2> $OUT/inflate_$v.err || { tail -20 $OUT/inflate_$v.err; exit 1; }
  else timeout -k 10 200 python -u tools/ab_run.py $v.so tools/inflate_bench.py > $OUT/inflate_$v.json 2> $OUT/inflate_$v.err || { tail -20 $OUT/inflate_$v.err; exit 1; }; fi
  python -c "import json;d=json.load(open('$OUT/inflate_$v.json'));print('$v', [round(r['kernel_ms'],2) for r in d['runs']], [r['bad_members'] for r in d['runs']], d['identical'])"
done
