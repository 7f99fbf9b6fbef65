#!/bin/bash
# build_variant.sh <kernels.hip> <out.so> : build a variant of the engine library for A/B timing
set -e
D=$(cd "$(dirname "$0")/.." && pwd)
C=$D/covid-spings-variant-caller_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I$D/include -I$C -o "$2" "$1" $C/spg_api.cpp
