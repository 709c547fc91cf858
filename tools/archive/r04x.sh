#!/bin/bash
# C5: per-launch hop table of the current build (folds on at 256 streams)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
bash $R/tools/c5_prof.sh r04x > $R/gpurun_out/r04x_c5prof.log 2>&1 || { echo "c5 prof failed"; exit 1; }
python $R/tools/c5_hop_table.py $R/gpurun_out/prof_r04x > $R/gpurun_out/r04x_c5_hop_table.txt && cat $R/gpurun_out/r04x_c5_hop_table.txt
