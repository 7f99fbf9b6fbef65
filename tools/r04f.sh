# r04f: finishing-ring width A/B (SPG_NB 4 vs 8 builds) at 1,000x (stacked) and 10,000x, list vs fused
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04f}; mkdir -p $OUT
V=$GRAFT_REPO_ROOT/tools/_variants/nb8/libspings_gpu.so
run() { # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --legs sars1k --reps 8 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -20 $OUT/$tag.err; exit 1; }
}
for r in 1 2; do
  run nb4_list_$r SPG_LIST=1
  run nb4_fused_$r SPG_LIST=0
  run nb8_list_$r SPG_LIST=1 SPG_GPU_LIB=$V
  run nb8_fused_$r SPG_LIST=0 SPG_GPU_LIB=$V
done
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    s = d["sars1k"]
    print(f.split("/")[-1], "main", round(d["roofline"]["kernel_ms"] * 1e3, 2), "us", round(d["roofline"]["frac"], 4),
          "| sars1k", round(s["ms_per_step"], 4), "ms", round(s["roofline"]["frac"], 4), round(s["roofline"]["kernel_ms"], 4), round(s["finalize_ms"], 4))
PY
echo done
