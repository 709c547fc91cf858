#!/bin/bash
# C5: LSTM step launched twice per layer (timing only): the second launch finds W in L2
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export CRN_MX_STEP_TWICE=1
bash $R/tools/c5_prof.sh r04y2 > $R/gpurun_out/r04y2_c5prof.log 2>&1 || { echo "c5 prof failed"; exit 1; }
python $R/tools/c5_hop_table.py $R/gpurun_out/prof_r04y2 > $R/gpurun_out/r04y2_c5_hop_table.txt && cat $R/gpurun_out/r04y2_c5_hop_table.txt
