# r04zn: end-to-end leg (tools/e2e_only.py: 4 BAMs through process_bam, 8 through process_bams, 10,000x, 16 host threads),
# records plans' parallel record scan: old (_lib/ab/pileup_old.so: its ranges ran on one thread) vs current (ranges on
# every thread, 8 chains stepped in turn per thread); then SPP_TIMING of the current one, and a lone process_bam with the
# parallel scan after the host inflate (SPP_PAR_SCAN=1)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04zn}; mkdir -p $OUT
L=$GRAFT_REPO_ROOT/covid-spings-variant-caller_amd/_lib
for r in 1 2; do
  for v in old cur par; do
    unset SPP_PILEUP_LIB SPP_PAR_SCAN
    [ $v = old ] && export SPP_PILEUP_LIB=$L/ab/pileup_old.so
    [ $v = par ] && export SPP_PAR_SCAN=1
    timeout -k 10 300 python3 -u tools/e2e_only.py 4 0 16 > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { echo "$v failed"; tail -20 $OUT/${v}_$r.err; exit 1; }
    python3 - $OUT/${v}_$r.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], {k: (round(d[k]["process_bams"]["positions_per_s_per_bam"]), round(d[k]["positions_per_s_per_bam"])) for k in ("uncapped", "parity_mode_max_depth_8000")})
PY
  done
done
unset SPP_PILEUP_LIB SPP_PAR_SCAN
SPP_TIMING=1 timeout -k 10 300 python3 -u tools/e2e_only.py 4 0 16 > $OUT/timing.json 2> $OUT/timing.err || { echo "timing failed"; exit 1; }
grep "spp timing" $OUT/timing.err | tail -16 | cut -c1-220
