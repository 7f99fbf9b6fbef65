# r04zi: per-XCD ends of the deep kernel with its block->work mapping rotated (SPG_WAVE_ROT): does the slow XCD
# follow the work or stay put?
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04zi}; mkdir -p $OUT
for r in 0 1 4 0; do
  SPG_WAVE_ROT=$r timeout -k 10 200 python3 -u tools/wavetimes.py 10000 $OUT/wt_rot$r.json > $OUT/wt_rot$r.log 2>&1 || { echo "wt $r failed"; tail -10 $OUT/wt_rot$r.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/wt_rot$r.json')); print('rot $r span', d['span_us']); [print(' ', l) for l in d['per_xcc_end_us_every_launch']]"
done
