#!/bin/bash
# C5 fused kernels with transposed-accumulator epilogues
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_crn.py $R/tests/test_gpu_crn_nlms.py -k "fused_stream or fp8 or stream" -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r04r_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r04r_tests.log; exit 1; }
tail -1 $R/gpurun_out/r04r_tests.log
bash $R/tools/c5_ab_env.sh 3 AEC_CRN_STREAM_FUSE=15 || exit 1
