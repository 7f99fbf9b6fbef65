set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/kb.log
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for fb in 64 256 128; do
  SPG_FIN_BLOCK=$fb timeout -k 10 200 python tools/kbench.py --tag fb$fb 2>/dev/null >> gpurun_out/kb.log
done
cut -c1-200 gpurun_out/kb.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
bash tools/prof_bench.sh gpurun_out/prof_r01
ls -R gpurun_out/prof_r01 | head -40
