#!/bin/bash
# g11.sh: A/B of prefetch depth / load policy variants, then PMC passes of the in-tree kernel
cd /root/repo
export TMPDIR=/tmp
VARIANTS="A B C D E" DEPTHS="10000 1000" bash tools/gab.sh || exit 1
bash tools/pmc.sh gpurun_out/pmc11
