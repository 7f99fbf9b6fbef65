set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 1000 python bench.py --workload chr1_30x --no-e2e --no-cpu-baseline --steps 20 --warmup 2 > gpurun_out/bench_chr1.json 2> gpurun_out/bench_chr1.err || { tail -30 gpurun_out/bench_chr1.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_chr1.json')); print(d['metric'], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['finalize_ms'], d['datagen_s'])"
