#!/bin/bash
# round 5 batch d: the 16-wave NLMS analysis kernel (AEC_NLMS_K16=1): bit-exactness tests, C2 A/B
# against the 12-wave kernel, its tick profile
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_nlms.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_stream.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r05d_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $O/r05d_tests.log | head -20; tail -5 $O/r05d_tests.log; exit 1; }
tail -1 $O/r05d_tests.log
bash $R/tools/env_ab.sh AEC_NLMS_K16 "0 1" 3 > $O/r05d_k16.log 2>&1 || { echo "k16 ab failed"; tail $O/r05d_k16.log; exit 1; }
cat $O/r05d_k16.log
AEC_NLMS_K16=1 AEC_HIP_LIB=$R/acoustic-echo-cancellation_amd/aec_amd/ab/tick.so timeout -k 10 120 python $R/tools/tick_prof.py > $O/r05d_nlms16_tick.txt 2>&1 || { echo "tick prof failed"; tail $O/r05d_nlms16_tick.txt; exit 1; }
head -20 $O/r05d_nlms16_tick.txt
