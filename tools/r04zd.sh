# r04zd: SQ counters of k_inflate (LDS-table decoder) vs the token-batch variant (_lib/ab/inflate_batch.so)
cd $GRAFT_REPO_ROOT
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/${1:-r04zd}; mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_BRANCH"
for v in base batch; do
  if [ $v = batch ]; then export SPG_GPU_LIB=$ROOT/covid-spings-variant-caller_amd/_lib/ab/inflate_batch.so; else unset SPG_GPU_LIB; fi
  i=0
  for pass in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pass -d $OUT/${v}_pmc$i -o run --output-format csv -- python3 $ROOT/tools/inflate_bench.py > $OUT/${v}_pmc$i.log 2>&1 || { echo "$v pass $i failed"; tail -5 $OUT/${v}_pmc$i.log; exit 1; }
  done
done
python3 $ROOT/tools/pmc_sum.py $OUT k_inflate
