# r04zo: end-to-end leg (tools/e2e_only.py), process_bams: concurrent GPU inflate calls per device (SPG_INFLATE_SLOTS
# 1 / 2) x concurrent plans (SPG_PLAN_WORKERS 2 / 3), 2 rounds
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04zo}; mkdir -p $OUT
for r in 1 2; do
  for v in s1w2 s2w2 s1w3 s2w3; do
    export SPG_INFLATE_SLOTS=${v:1:1} SPG_PLAN_WORKERS=${v:3:1}
    timeout -k 10 300 python3 -u tools/e2e_only.py 4 0 16 > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { echo "$v failed"; tail -20 $OUT/${v}_$r.err; exit 1; }
    python3 - $OUT/${v}_$r.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], {k: (round(d[k]["process_bams"]["positions_per_s_per_bam"]), round(d[k]["positions_per_s_per_bam"])) for k in ("uncapped", "parity_mode_max_depth_8000")})
PY
  done
done
