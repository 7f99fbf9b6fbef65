#!/bin/bash
# r05zq: the lone process_bam's BAM goes up in 16 MiB ranges while the file is read (spp_bam_map_begin / _read / _finish
# + spg_bam_upload_range / _members) — device-pileup, live-caller and live-loop GPU tests, then the end-to-end leg
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zq}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_device_pileup_gpu.py tests/test_live_caller_gpu.py tests/test_live_loop_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python3 -u bench.py --legs e2e --reps 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read().strip().splitlines()[-1])
for tag, e in d.get("end_to_end", {}).items():
    if not isinstance(e, dict) or "breakdown_one_bam_device" not in e: continue
    print(tag, "lone process_bam positions/s per BAM %.4g" % e["positions_per_s_per_bam"], "s_per_bam %.4f" % e["s_per_bam"])
    print("   breakdown", {k: round(v, 2) for k, v in e["breakdown_one_bam_device"].items()})
    print("   process_bams %.4g" % e["process_bams"]["positions_per_s_per_bam"])
    for k in ("vcqueue_loop", "vcqueue_loop_write_behind"):
        v = e.get(k)
        if v: print("  ", k, {a: v[a] for a in ("ms_per_bam", "process_bam_ms", "create_checkpoint_ms", "write_vcf_ms")})
PY
