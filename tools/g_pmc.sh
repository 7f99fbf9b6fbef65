#!/bin/bash
# g_pmc.sh: PMC passes over kbench for each variant in VARIANTS -> gpurun_out/pmc_<v>
cd /root/repo
for v in ${VARIANTS:-B}; do
  SPG_GPU_LIB=/root/repo/tools/_variants/lib_$v.so bash tools/pmc.sh gpurun_out/pmc_$v || exit 1
done
