#!/bin/bash
# C3 kernel traces (bf16 and fp8) of the current build
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
bash $R/tools/crn_prof.sh r04ae_bf16 || exit 1
bash $R/tools/crn_prof.sh r04ae_fp8 --dtype fp8 || exit 1
for t in bf16 fp8; do
  python $R/tools/crn_kstats.py $R/gpurun_out/prof_r04ae_$t > $R/gpurun_out/r04ae_${t}_kernel_table.txt 2>&1 || exit 1
  head -16 $R/gpurun_out/r04ae_${t}_kernel_table.txt
done
