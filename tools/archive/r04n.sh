#!/bin/bash
# static-shape fused conv levels (batch and per-hop): bit-exact tests, C3 probe, C5 hop time, trace
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_crn.py $R/tests/test_gpu_crn_nlms.py -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r04n_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r04n_tests.log; exit 1; }
tail -1 $R/gpurun_out/r04n_tests.log
bash $R/tools/crn_ab.sh AEC_CRN_BATCH_DEC "0 1" || exit 1
bash $R/tools/c5_ab_env.sh 2 AEC_CRN_STREAM_FUSE=7 AEC_CRN_STREAM_FUSE=0 || exit 1
bash $R/tools/crn_prof.sh r04n || exit 1
python $R/tools/crn_kstats.py $R/gpurun_out/prof_r04n > $R/gpurun_out/r04n_crn_kernel_table.txt && head -12 $R/gpurun_out/r04n_crn_kernel_table.txt
