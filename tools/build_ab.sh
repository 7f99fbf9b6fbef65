#!/bin/bash
# build_ab.sh <name> [SRC=<source>] <hipcc flags...>: an A/B variant of libspings_gpu.so with one source (default
# spg_kernels.hip) rebuilt under the given flags (e.g. -DSPG_INFLATE_LANE), the other objects shared with the in-tree
# build -> _lib/ab/<name>.so.  Load it with tools/ab_run.py <name>.so <script> [args] (the product has no library-swap
# environment variable).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
L=$ROOT/covid-spings-variant-caller_amd/_lib
N=$1; shift
SRC=spg_kernels.hip
if [[ "$1" == SRC=* ]]; then SRC=${1#SRC=}; shift; fi
mkdir -p $L/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include "$@" -c $ROOT/covid-spings-variant-caller_amd/csrc/$SRC \
  -o $L/ab/$N.var.o -Rpass-analysis=kernel-resource-usage 2> $L/ab/$N.remarks
OBJS=""
for o in spg_kernels.hip spg_tile.hip spg_lite.hip spg_fill.hip spg_inflate.hip spg_ckpt.hip spg_bam.hip spg_plan.hip spg_api.cpp spg_multi.cpp; do
  [ "$o" = "$SRC" ] || OBJS="$OBJS $L/obj/$o.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-z,defs -o $L/ab/$N.so $L/ab/$N.var.o $OBJS -lrccl
