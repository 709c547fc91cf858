#!/bin/bash
# round 5 batch c: NLMS / fused-synthesis GPU tests (ERB bins in registers, role-placement knobs),
# A/B tree (ERB bins in registers) vs ab/magrow.so, gru_synth role priority / placement sweep,
# NLMS tick profile of the tree
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_nlms.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_stream.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r05c_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $O/r05c_tests.log | head -20; tail -5 $O/r05c_tests.log; exit 1; }
tail -1 $O/r05c_tests.log
bash $R/tools/libs_ab.sh 3 tree acoustic-echo-cancellation_amd/aec_amd/ab/magrow.so > $O/r05c_ab.log 2>&1 || { echo "ab failed"; tail $O/r05c_ab.log; exit 1; }
cat $O/r05c_ab.log
bash $R/tools/env_ab.sh AEC_FUSED_MODE "0 16384 24576 8192 12288 40 20480" 2 > $O/r05c_fmode.log 2>&1 || { echo "fmode ab failed"; tail $O/r05c_fmode.log; exit 1; }
cat $O/r05c_fmode.log
AEC_HIP_LIB=$R/acoustic-echo-cancellation_amd/aec_amd/ab/tick.so timeout -k 10 120 python $R/tools/tick_prof.py > $O/r05c_nlms_tick.txt 2>&1 || { echo "tick prof failed"; exit 1; }
head -14 $O/r05c_nlms_tick.txt
