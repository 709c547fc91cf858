#!/bin/bash
# round-4 session-2 A/B batch: new batch-encoder test, GRU streams per block, GEMM tile order
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_crn.py -k "batch_enc or back_mask" -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r04j_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r04j_tests.log; exit 1; }
tail -2 $R/gpurun_out/r04j_tests.log
bash $R/tools/env_ab.sh AEC_GRU_NS "1 2" 2 || exit 1
bash $R/tools/crn_ab.sh AEC_CRN_BATCH_ENC "0 1" || exit 1
bash $R/tools/xcd_ab.sh "0 4 8" 1 || exit 1
