#!/bin/bash
# round 5 batch b: GPU suite with the tightened bars and the scalar NLMS recursion, A/B of the
# C2 line (tree = scalar NLMS + |E| rows, ab/scalar.so = scalar NLMS only, ab/base.so = packed NLMS), tick profiles of both C2 kernels
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 240 --timeout-method thread -s > $O/r05b_gputest.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $O/r05b_gputest.log | head -20; tail -5 $O/r05b_gputest.log; exit 1; }
tail -1 $O/r05b_gputest.log
cp $O/parity_margins.json $O/r05b_parity_margins.json
bash $R/tools/libs_ab.sh 3 tree acoustic-echo-cancellation_amd/aec_amd/ab/scalar.so acoustic-echo-cancellation_amd/aec_amd/ab/base.so > $O/r05b_ab.log 2>&1 || { echo "ab failed"; tail $O/r05b_ab.log; exit 1; }
cat $O/r05b_ab.log
AEC_HIP_LIB=$R/acoustic-echo-cancellation_amd/aec_amd/ab/tick.so timeout -k 10 120 python $R/tools/tick_prof.py > $O/r05b_nlms_tick.txt 2>&1 || { echo "tick prof failed"; exit 1; }
AEC_HIP_LIB=$R/acoustic-echo-cancellation_amd/aec_amd/ab/tick.so timeout -k 10 120 python $R/tools/gru_tick_prof.py > $O/r05b_gru_tick.txt 2>&1 || { echo "gru tick prof failed"; tail $O/r05b_gru_tick.txt; exit 1; }
head -14 $O/r05b_nlms_tick.txt; cat $O/r05b_gru_tick.txt
