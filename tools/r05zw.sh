#!/bin/bash
# r05zw: checkpoint shards whose large arrays go out in four files at once — checkpoint GPU tests, then the e2e leg (VCQueue loops)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r05zw}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_live_caller_gpu.py tests/test_live_loop_gpu.py tests/test_multi_gpu.py tests/test_ckpt_compact_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python3 -u bench.py --legs e2e --reps 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read().strip().splitlines()[-1])
for tag, e in d.get("end_to_end", {}).items():
    if not isinstance(e, dict): continue
    for k in ("vcqueue_loop", "vcqueue_loop_write_behind"):
        v = e.get(k)
        if v: print(tag, k, {a: v[a] for a in ("ms_per_bam", "process_bam_ms", "create_checkpoint_ms", "write_vcf_ms", "per_bam_ms", "checkpoint_shard_mb")})
PY
