#!/bin/bash
# C5 fold variants as separate instantiations: stream tests, then folds against stream count
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_crn.py $R/tests/test_gpu_crn_nlms.py -k "fused_stream or fp8 or stream" -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r04v_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r04v_tests.log; exit 1; }
tail -1 $R/gpurun_out/r04v_tests.log
bash $R/tools/r04u.sh
