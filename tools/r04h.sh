# r04h: end-to-end host plan A/B on the box: threads 16 / 32 x record scan parallel / serial; nproc and cgroup CPU quota
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04h}; mkdir -p $OUT
nproc > $OUT/cpu.txt; cat /sys/fs/cgroup/cpu.max >> $OUT/cpu.txt 2>/dev/null; python3 -c "import os; print(len(os.sched_getaffinity(0)))" >> $OUT/cpu.txt
for r in 1 2; do
  for cfg in "16 1" "16 0" "32 1" "32 0"; do
    set -- $cfg
    SPP_PAR_SCAN=$2 SPP_TIMING=1 timeout -k 10 200 python3 -u tools/e2e_only.py 4 0 $1 > $OUT/e2e_$1_$2_$r.json 2> $OUT/e2e_$1_$2_$r.err || { echo "e2e $cfg failed"; tail -20 $OUT/e2e_$1_$2_$r.err; exit 1; }
  done
done
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/e2e_*.json")):
    d = json.loads(open(f).read())
    print(f.split("/")[-1], {k: (round(d[k]["positions_per_s_per_bam"]), round(d[k]["breakdown_one_bam"]["host_plan_records_s"] * 1e3, 1))
                             for k in ("uncapped", "parity_mode_max_depth_8000")})
PY
cat $OUT/cpu.txt
