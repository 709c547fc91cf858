#!/bin/bash
# C5: LSTM layer step with both cells per workgroup (AEC_CRN_MX_PAIR): bit-identity, then A/B and hop table
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_crn.py -k "mx_scale_paths" -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r04aa_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r04aa_tests.log; exit 1; }
tail -1 $R/gpurun_out/r04aa_tests.log
bash $R/tools/c5_ab_env.sh 3 AEC_CRN_MX_PAIR=0 AEC_CRN_MX_PAIR=1 || exit 1
export AEC_CRN_MX_PAIR=1
bash $R/tools/c5_prof.sh r04aa > $R/gpurun_out/r04aa_c5prof.log 2>&1 || { echo "c5 prof failed"; exit 1; }
python $R/tools/c5_hop_table.py $R/gpurun_out/prof_r04aa > $R/gpurun_out/r04aa_c5_hop_table.txt && cat $R/gpurun_out/r04aa_c5_hop_table.txt
