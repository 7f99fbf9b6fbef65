# r04zl: end-to-end leg (tools/e2e_only.py: 4 BAMs through process_bam, 8 through process_bams, 10,000x, 16 host threads),
# GPU inflate calls of concurrent plans serialised (SPG_INFLATE_SLOTS=1, the r04zg form) vs overlapped (2 slots, default)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04zl}; mkdir -p $OUT
for r in 1 2; do
  for v in 1 2; do
    SPG_INFLATE_SLOTS=$v timeout -k 10 300 python3 -u tools/e2e_only.py 4 0 16 > $OUT/slots${v}_$r.json 2> $OUT/slots${v}_$r.err || { echo "slots $v failed"; tail -20 $OUT/slots${v}_$r.err; exit 1; }
    python3 - $OUT/slots${v}_$r.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("slots", sys.argv[2], {k: (round(d[k]["process_bams"]["positions_per_s_per_bam"]), round(d[k]["positions_per_s_per_bam"])) for k in ("uncapped", "parity_mode_max_depth_8000")})
PY
  done
done
SPP_TIMING=1 timeout -k 10 300 python3 -u tools/e2e_only.py 4 0 16 > $OUT/timing.json 2> $OUT/timing.err || { echo "timing failed"; exit 1; }
grep "gpu inflate" $OUT/timing.err | tail -12
