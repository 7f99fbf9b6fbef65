#!/bin/bash
# r05a: spg_multi device-slice path + checkpoint compaction / VCQueue-named checkpoints (tests), then bench --gpus 2
# without a launcher (gloo, one GPU standing in for two) and the N=1 multi leg
set -o pipefail
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_multi_gpu.py tests/test_ckpt_compact_gpu.py tests/test_live_caller_gpu.py > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --legs none --reps 5 > $OUT/bench_g2.json 2> $OUT/bench_g2.err || { tail -30 $OUT/bench_g2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_g2.json'));print(d['n_gpus'],d['config']['parallelism'],d['value'],d['ms_per_step'],d['config']['ranks']);m=d.get('multi_device');print({k:m.get(k) for k in ('devices','rccl','value','ms_per_step','kernel_ms_slowest_device','error','calls_per_step')})"
timeout -k 10 400 python -u bench.py --legs multi --reps 5 > $OUT/bench_g1.json 2> $OUT/bench_g1.err || { tail -30 $OUT/bench_g1.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_g1.json'));print(d['n_gpus'],d['value'],d['ms_per_step'],d['roofline']['frac']);m=d.get('multi_device');print({k:m.get(k) for k in ('devices','rccl','value','ms_per_step','kernel_ms_slowest_device','error')})"
