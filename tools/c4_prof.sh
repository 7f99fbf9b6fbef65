#!/bin/bash
# c4_prof.sh <outdir>: BASELINE config 4 (10,000 SARS-CoV-2 BAMs x 100x) — the bench's config4 line with its live
# per-BAM form, then a kernel-trace summary and the FETCH_SIZE / WRITE_SIZE passes of the same command.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/${1:-gpurun_out/c4}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
B="$ROOT/bench.py --no-cpu-baseline --no-e2e --no-parity --no-chr1 --reps ${REPS:-5} --steps 3 --warmup 2 ${EXTRA:-}"
timeout -k 10 400 python3 -u $B > $OUT/bench.log 2>&1 || { echo "bench failed" >> $OUT/fail.log; exit 1; }
P="$ROOT/bench.py --no-cpu-baseline --no-e2e --no-parity --no-chr1 --reps 1 --steps 1 --warmup 1 --min-ms 1 ${EXTRA:-}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 -u $P > $OUT/trace.log 2>&1 || { echo "trace failed" >> $OUT/fail.log; exit 1; }
python3 $ROOT/tools/prof_filter.py $OUT/trace
i=0
for pass in FETCH_SIZE WRITE_SIZE ${SQ:+"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"}; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $pass -d $OUT/pmc$i -o run --output-format csv -- python3 -u $P > $OUT/pmc$i.log 2>&1 || { echo "pmc $pass failed" >> $OUT/fail.log; exit 1; }
  python3 $ROOT/tools/prof_filter.py $OUT/pmc$i
done
