# r04z: per-XCD end times of the deep kernel over several launches and two processes (is the slow XCD fixed?)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04z}; mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 200 python3 -u tools/wavetimes.py 10000 $OUT/wt_$r.json > $OUT/wt_$r.log 2>&1 || { echo "wt $r failed"; tail -10 $OUT/wt_$r.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/wt_$r.json')); print('span', d['span_us']); [print(l) for l in d['per_xcc_end_us_every_launch']]"
done
