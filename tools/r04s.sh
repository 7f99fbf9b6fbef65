# r04s: end-to-end host plan phases on the box (32 threads; record scan parallel vs serial), CPU share
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04s}; mkdir -p $OUT
nproc > $OUT/cpu.txt; cat /sys/fs/cgroup/cpu.max >> $OUT/cpu.txt 2>/dev/null; python3 -c "import os; print(len(os.sched_getaffinity(0)))" >> $OUT/cpu.txt
lscpu | head -20 >> $OUT/cpu.txt
for cfg in "32 1" "32 0" "64 1"; do
  set -- $cfg
  SPP_PAR_SCAN=$2 SPP_TIMING=1 timeout -k 10 200 python3 -u tools/e2e_only.py 4 0 $1 > $OUT/e2e_$1_$2.json 2> $OUT/e2e_$1_$2.err || { echo "e2e $cfg failed"; tail -20 $OUT/e2e_$1_$2.err; exit 1; }
done
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/e2e_*.json")):
    d = json.loads(open(f).read())
    print(f.split("/")[-1], {k: (round(d[k]["positions_per_s_per_bam"]), round(d[k]["breakdown_one_bam"]["host_plan_records_s"] * 1e3, 1))
                             for k in ("uncapped", "parity_mode_max_depth_8000")})
PY
grep -h "spp" $OUT/e2e_32_1.err | head -30
cat $OUT/cpu.txt | head -8
