set -e
cd /root/repo
export TMPDIR=/tmp
for v in BASE NOREPLAY; do
SPG_GPU_LIB=tools/_variants/lib$v.so timeout -k 10 200 python tools/kbench.py --tag $v 2>/dev/null | cut -c1-150
done
