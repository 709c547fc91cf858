#!/bin/bash
# C5: stage buffers of the small MX GEMM tile (CRN_MX_SMALL_NBUF 2 / 3 / 4), then the hop table at the best
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
bash $R/tools/c5_ab_env.sh 2 CRN_MX_SMALL_NBUF=2 CRN_MX_SMALL_NBUF=3 CRN_MX_SMALL_NBUF=4 || exit 1
export CRN_MX_SMALL_NBUF=4
bash $R/tools/c5_prof.sh r04y > $R/gpurun_out/r04y_c5prof.log 2>&1 || { echo "c5 prof failed"; exit 1; }
python $R/tools/c5_hop_table.py $R/gpurun_out/prof_r04y > $R/gpurun_out/r04y_c5_hop_table.txt && cat $R/gpurun_out/r04y_c5_hop_table.txt
