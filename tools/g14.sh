#!/bin/bash
# g14.sh: middle-chunk fast path A/B (all variants with nt loads)
cd /root/repo
export TMPDIR=/tmp
VARIANTS="A0 F1 F2 F3" DEPTHS="10000 1000" bash tools/gab.sh || exit 1
