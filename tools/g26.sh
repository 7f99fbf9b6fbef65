#!/bin/bash
# g26.sh: the N > 1 bench path on one GPU (gloo, 2 ranks), then the chr1 30x workload
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/b2.json 2> gpurun_out/b2.err || { tail -20 gpurun_out/b2.err; exit 1; }
cat gpurun_out/b2.json
timeout -k 10 600 python bench.py --workload chr1_30x --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bchr1.json 2> gpurun_out/bchr1.err || { tail -20 gpurun_out/bchr1.err; exit 1; }
cat gpurun_out/bchr1.json
