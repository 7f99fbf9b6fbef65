#!/bin/bash
# inflate_ab_run.sh <outdir> <variant>...: tools/inflate_bench.py (the 10,000x BAM's BGZF members through
# spg_bgzf_inflate: kernel ms, identity vs gzip) on the in-tree library ("default") and on A/B builds of
# tools/src_ab.py (_lib/ab/<variant>.so), interleaved twice.  Each run under its own limit; stops at the first failure.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/$1
shift
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then
      timeout -k 10 300 python3 tools/inflate_bench.py > $OUT/${v}_$round.json 2> $OUT/${v}_$round.err || exit 1
    else
      timeout -k 10 300 python3 tools/ab_run.py $v.so tools/inflate_bench.py > $OUT/${v}_$round.json 2> $OUT/${v}_$round.err || exit 1
    fi
  done
done
