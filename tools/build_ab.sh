#!/bin/bash
# build_ab.sh <name> <hipcc flags...>: an A/B variant of libspings_gpu.so with spg_kernels.hip rebuilt under the given
# flags (e.g. -DSPG_CLIP=1), the other objects shared with the in-tree build -> _lib/ab/<name>.so (SPG_GPU_LIB=...)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
L=$ROOT/covid-spings-variant-caller_amd/_lib
N=$1; shift
mkdir -p $L/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include "$@" -c $ROOT/covid-spings-variant-caller_amd/csrc/spg_kernels.hip \
  -o $L/ab/$N.kernels.o -Rpass-analysis=kernel-resource-usage 2> $L/ab/$N.remarks
OBJS=""
for o in spg_tile.hip spg_lite.hip spg_fill.hip spg_inflate.hip spg_api.cpp spg_multi.cpp; do OBJS="$OBJS $L/obj/$o.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-z,defs -o $L/ab/$N.so $L/ab/$N.kernels.o $OBJS -lrccl
grep -A12 "k_acc_segILi4ELb1ELi4ELb1ELb1E" $L/ab/$N.remarks | grep -E "VGPRs:|SGPRs Spill|VGPRs Spill|ScratchSize|Occupancy" | head -6
