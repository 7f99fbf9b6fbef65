set -e
cd /root/repo
export TMPDIR=/tmp
rm -rf gpurun_out/prof_r01
bash tools/prof_bench.sh gpurun_out/prof_r01
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-200 gpurun_out/bench.json
