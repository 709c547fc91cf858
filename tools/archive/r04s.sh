#!/bin/bash
# C5: encoder level 4 (MX) folded into the fused front
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_crn.py $R/tests/test_gpu_crn_nlms.py -k "fused_stream or fp8 or stream" -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r04s_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r04s_tests.log; exit 1; }
tail -1 $R/gpurun_out/r04s_tests.log
bash $R/tools/c5_ab_env.sh 2 AEC_CRN_STREAM_FUSE=15 AEC_CRN_STREAM_FUSE=31 || exit 1
bash $R/tools/c5_prof.sh r04s > $R/gpurun_out/r04s_c5prof.log 2>&1 || { echo "c5 prof failed"; exit 1; }
python $R/tools/c5_hop_table.py $R/gpurun_out/prof_r04s > $R/gpurun_out/r04s_c5_hop_table.txt && cat $R/gpurun_out/r04s_c5_hop_table.txt
