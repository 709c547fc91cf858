#!/bin/bash
# padded LDS maps in the C5 fused kernels + batch encoder FR variants
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_crn.py -k "batch_enc or fused_stream or streaming_equals or mx_scale" -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r04l_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r04l_tests.log; exit 1; }
tail -1 $R/gpurun_out/r04l_tests.log
bash $R/tools/crn_ab.sh AEC_CRN_ENC_FR "2 4 8" || exit 1
bash $R/tools/c5_ab_env.sh 2 AEC_CRN_STREAM_FUSE=7 || exit 1
