#!/bin/bash
# round 5 batch e: the ref waves' two ERB projections in one pass (erb_project2): bit-exactness tests,
# C2 A/B against two passes (AEC_NLMS_MODE=16), tick profile
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_nlms.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_stream.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r05e_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $O/r05e_tests.log | head -20; tail -5 $O/r05e_tests.log; exit 1; }
tail -1 $O/r05e_tests.log
bash $R/tools/env_ab.sh AEC_NLMS_MODE "0 16" 3 > $O/r05e_erb2.log 2>&1 || { echo "ab failed"; tail $O/r05e_erb2.log; exit 1; }
cat $O/r05e_erb2.log
AEC_HIP_LIB=$R/acoustic-echo-cancellation_amd/aec_amd/ab/tick.so timeout -k 10 120 python $R/tools/tick_prof.py > $O/r05e_nlms_tick.txt 2>&1 || { echo "tick prof failed"; tail $O/r05e_nlms_tick.txt; exit 1; }
head -14 $O/r05e_nlms_tick.txt
