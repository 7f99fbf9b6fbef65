# r04zp: a lone process_bam (tools/e2e_only.py's 4-BAM stream) with the host inflate (default) vs the GPU inflater
# (SPG_GPU_INFLATE=1) now that the scan after a GPU inflate runs on every thread; 3 rounds
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04zp}; mkdir -p $OUT
for r in 1 2 3; do
  for v in host gpu; do
    unset SPG_GPU_INFLATE
    [ $v = gpu ] && export SPG_GPU_INFLATE=1
    timeout -k 10 300 python3 -u tools/e2e_only.py 4 0 16 > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { echo "$v failed"; tail -20 $OUT/${v}_$r.err; exit 1; }
    python3 - $OUT/${v}_$r.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], {k: (round(d[k]["process_bams"]["positions_per_s_per_bam"]), round(d[k]["positions_per_s_per_bam"])) for k in ("uncapped", "parity_mode_max_depth_8000")})
PY
  done
done
