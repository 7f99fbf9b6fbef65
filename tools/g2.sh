set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 3 --backend gloo > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2.err || { tail -30 gpurun_out/bench_n2.err; exit 1; }
cut -c1-600 gpurun_out/bench_n2_gloo.json
timeout -k 10 600 python bench.py --no-e2e --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['finalize_ms'])"
