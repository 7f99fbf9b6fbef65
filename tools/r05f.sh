#!/bin/bash
# r05f: the full GPU suite, then the e2e leg (pread map, raw checkpoint shards)
set -o pipefail
OUT=gpurun_out/r05f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/tests.txt 2>&1 || { tail -60 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
SPP_TIMING=1 timeout -k 10 600 python -u bench.py --no-main --legs e2e --e2e-many 16 > $OUT/e2e.json 2> $OUT/e2e.err || { tail -40 $OUT/e2e.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r05f/e2e.json"))["end_to_end"]
for tag in ("parity_mode_max_depth_8000", "uncapped"):
    e = d[tag]
    print(tag, "device %.3g" % e["positions_per_s_per_bam"], "records %.3g" % e["records_plan_path"]["positions_per_s_per_bam"],
          "host %.3g" % e["host_fill_path"]["positions_per_s_per_bam"], "process_bams %.3g" % e["process_bams"]["positions_per_s_per_bam"])
    print("  breakdown", {k: round(v, 2) if isinstance(v, float) else v for k, v in e["breakdown_one_bam_device"].items()})
    v = e["vcqueue_loop"]
    print("  vcqueue", {k: v[k] for k in ("ms_per_bam", "process_bam_ms", "create_checkpoint_ms", "write_vcf_ms", "checkpoint_shard_mb_per_bam")})
v = d["config4_process_bams"]["vcqueue_loop"]
print("config4 vcqueue", {k: v[k] for k in ("ms_per_bam", "process_bam_ms", "create_checkpoint_ms", "write_vcf_ms")})
PY
