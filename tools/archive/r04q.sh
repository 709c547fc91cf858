#!/bin/bash
# C5: decoder cl = 4 (MX) folded into the fused back
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_crn.py $R/tests/test_gpu_crn_nlms.py -k "fused_stream or fp8 or stream" -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r04q_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r04q_tests.log; exit 1; }
tail -1 $R/gpurun_out/r04q_tests.log
bash $R/tools/c5_ab_env.sh 2 AEC_CRN_STREAM_FUSE=7 AEC_CRN_STREAM_FUSE=15 || exit 1
bash $R/tools/c5_prof.sh r04q > $R/gpurun_out/r04q_c5prof.log 2>&1 || { echo "c5 prof failed"; exit 1; }
python $R/tools/c5_hop_table.py $R/gpurun_out/prof_r04q > $R/gpurun_out/r04q_c5_hop_table.txt && cat $R/gpurun_out/r04q_c5_hop_table.txt
bash $R/tools/inflight_ab.sh "2 3" 2 || exit 1
