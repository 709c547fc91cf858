#!/bin/bash
# transposed-accumulator epilogues in the batch fused kernels
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_crn.py -k "batch_fused or back_mask or ragged or streaming_equals" -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r04o_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r04o_tests.log; exit 1; }
tail -1 $R/gpurun_out/r04o_tests.log
bash $R/tools/crn_prof.sh r04o || exit 1
python $R/tools/crn_kstats.py $R/gpurun_out/prof_r04o > $R/gpurun_out/r04o_crn_kernel_table.txt && head -8 $R/gpurun_out/r04o_crn_kernel_table.txt
