#!/bin/bash
# r05zs: host worker pool — device-pileup / live-caller / plan GPU tests, the end-to-end leg, and the process_bam(s)
# GPU-busy timeline with the host plan's stage times
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zs}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_device_pileup_gpu.py tests/test_live_caller_gpu.py tests/test_live_loop_gpu.py tests/test_records_plan.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python3 -u bench.py --legs e2e --reps 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read().strip().splitlines()[-1])
for tag, e in d.get("end_to_end", {}).items():
    if not isinstance(e, dict) or "breakdown_one_bam_device" not in e: continue
    print(tag, "lone process_bam positions/s per BAM %.4g" % e["positions_per_s_per_bam"], "s_per_bam %.4f" % e["s_per_bam"])
    print("   breakdown", {k: round(v, 2) for k, v in e["breakdown_one_bam_device"].items()})
    print("   process_bams %.4g" % e["process_bams"]["positions_per_s_per_bam"], "records plan %.4g" % e["records_plan_path"]["positions_per_s_per_bam"])
    for k in ("vcqueue_loop", "vcqueue_loop_write_behind"):
        v = e.get(k)
        if v: print("  ", k, {a: round(v[a], 2) for a in ("ms_per_bam", "process_bam_ms", "create_checkpoint_ms", "write_vcf_ms")})
c4 = d.get("end_to_end", {}).get("config4_process_bams")
if c4: print("config4 process_bams positions/s %.4g" % c4["positions_per_s"], "s_per_bam", round(c4["s_per_bam"] * 1e3, 3), "ms")
PY
bash tools/r05zr.sh ${1:-r05zs}/tl | tail -30
