# r04w: same-box interleaved A/B of the deep kernel's load path: r04r (VGPR chunk addresses, LDS descriptors),
# r04t (soffset + lane descriptors), current (r04t + a round of three chunks with no exit in between); main + parity
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04w}; mkdir -p $OUT
L=$GRAFT_REPO_ROOT/covid-spings-variant-caller_amd/_lib
B="bench.py --legs parity --no-cpu-baseline --reps 10"
for r in 1 2 3; do
  for v in r04r r04t cur; do
    if [ $v = cur ]; then lib=$L/libspings_gpu.so; else lib=$L/ab/libspings_gpu_$v.so; fi
    SPG_GPU_LIB=$lib timeout -k 10 200 python3 -u $B > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { echo "$v failed"; tail -5 $OUT/${v}_$r.err; exit 1; }
    python3 - $OUT/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "main", round(d["ms_per_step"] * 1e3, 1), round(d["roofline"]["kernel_ms"] * 1e3, 1), "parity", round(d["parity_mode"]["ms_per_step"] * 1e3, 1), round(d["parity_mode"]["roofline"]["kernel_ms"] * 1e3, 1))
PY
  done
done
