# r04zm: the -m gpu suite on the xmix build, then a same-box interleaved A/B of the deep kernel's block -> work map
# (SPG_XMIX=0: identity, the r04zj form; 1: blocks 8k+j take work 8k+(j+k)%8), main + parity, 3 rounds; per-XCD ends
# with xmix (tools/wavetimes.py)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04zm}; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
B="bench.py --legs parity --no-cpu-baseline --reps 10"
for r in 1 2 3; do
  for v in 0 1; do
    SPG_XMIX=$v timeout -k 10 200 python3 -u $B > $OUT/xmix${v}_$r.json 2> $OUT/xmix${v}_$r.err || { echo "$v failed"; tail -5 $OUT/xmix${v}_$r.err; exit 1; }
    python3 - $OUT/xmix${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("xmix", sys.argv[2], "main", round(d["ms_per_step"] * 1e3, 1), round(d["roofline"]["kernel_ms"] * 1e3, 1), "parity", round(d["parity_mode"]["ms_per_step"] * 1e3, 1), round(d["parity_mode"]["roofline"]["kernel_ms"] * 1e3, 1))
PY
  done
done
for v in 1 0; do
  SPG_XMIX=$v timeout -k 10 200 python3 -u tools/wavetimes.py 10000 $OUT/wt_xmix$v.json > $OUT/wt_xmix$v.log 2>&1 || { echo "wt failed"; tail -10 $OUT/wt_xmix$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/wt_xmix$v.json')); print('xmix $v span', d['span_us'], 'resident', d['resident_waves_over_time'][-6:]); [print(' ', l) for l in d['per_xcc_end_us_every_launch']]"
done
