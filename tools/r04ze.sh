# r04ze: k_inflate at 5 waves/SIMD (96 VGPRs, _lib/ab/inflate_w5.so) vs the default (128 VGPRs, 4 waves), 2/3/4 members per block
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04ze}; mkdir -p $OUT
for v in w5 base; do
  if [ $v = w5 ]; then export SPG_GPU_LIB=$GRAFT_REPO_ROOT/covid-spings-variant-caller_amd/_lib/ab/inflate_w5.so; else unset SPG_GPU_LIB; fi
  for m in 2 3 4; do
    SPG_INFLATE_MPW=$m timeout -k 10 200 python3 -u tools/inflate_bench.py > $OUT/${v}_$m.json 2> $OUT/${v}_$m.err || { echo "bench $v $m failed"; tail -10 $OUT/${v}_$m.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/${v}_$m.json')); print('$v', $m, [round(r['kernel_ms'],1) for r in d['runs']], d['identical'])"
  done
done
