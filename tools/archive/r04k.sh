#!/bin/bash
# batch encoder front: bit-exact test, A/B, kernel trace
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_crn.py -k "batch_enc" -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r04k_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r04k_tests.log; exit 1; }
tail -1 $R/gpurun_out/r04k_tests.log
for r in 1 2; do bash $R/tools/crn_ab.sh AEC_CRN_BATCH_ENC "0 1" || exit 1; done
bash $R/tools/crn_prof.sh r04k || exit 1
python $R/tools/crn_kstats.py $R/gpurun_out/prof_r04k > $R/gpurun_out/r04k_crn_kernel_table.txt && head -14 $R/gpurun_out/r04k_crn_kernel_table.txt
