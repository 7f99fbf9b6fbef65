set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 3 --backend gloo > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2.err || { tail -30 gpurun_out/bench_n2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_n2_gloo.json')); print(d['n_gpus'], d['value'], d['ms_per_step'], d['calls_gathered_per_step'], d['candidates_per_gpu_step'], d['config'])"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 20 --warmup 2 --backend gloo > gpurun_out/bench_n4_gloo.json 2> gpurun_out/bench_n4.err || { tail -30 gpurun_out/bench_n4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_n4_gloo.json')); print(d['n_gpus'], d['value'], d['ms_per_step'], d['calls_gathered_per_step'])"
