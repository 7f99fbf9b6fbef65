"""Run only bench.py's end-to-end leg (dev tool): python tools/e2e_only.py [bams] [many] [threads]"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import spings  # noqa: E402,F401
import bench  # noqa: E402

args = types.SimpleNamespace(eff_depth=10000.0, e2e_bams=int(sys.argv[1]) if len(sys.argv) > 1 else 4,
                             e2e_many=int(sys.argv[2]) if len(sys.argv) > 2 else 0,
                             e2e_threads=int(sys.argv[3]) if len(sys.argv) > 3 else min(16, len(os.sched_getaffinity(0))))
print(json.dumps(bench.end_to_end(args, 0), indent=1), flush=True)
