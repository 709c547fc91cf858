#!/bin/bash
# batch decoder fusion: bit-exact tests, kernel trace
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_crn.py -k "batch_fused or back_mask" -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r04m_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r04m_tests.log; exit 1; }
tail -1 $R/gpurun_out/r04m_tests.log
bash $R/tools/crn_ab.sh AEC_CRN_BATCH_DEC "0 1" || exit 1
bash $R/tools/crn_prof.sh r04m || exit 1
python $R/tools/crn_kstats.py $R/gpurun_out/prof_r04m > $R/gpurun_out/r04m_crn_kernel_table.txt && head -16 $R/gpurun_out/r04m_crn_kernel_table.txt
