#!/bin/bash
# round 5 batch f: branch-free bin-256 |E| store, the gru_synth OLA on the gi waves (AEC_FUSED_MODE bit 15):
# tests, C2 A/B, tick profiles of both kernels
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_nlms.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_stream.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r05f_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $O/r05f_tests.log | head -20; tail -5 $O/r05f_tests.log; exit 1; }
tail -1 $O/r05f_tests.log
bash $R/tools/env_ab.sh AEC_FUSED_MODE "0 32768" 3 > $O/r05f_ola.log 2>&1 || { echo "ab failed"; tail $O/r05f_ola.log; exit 1; }
cat $O/r05f_ola.log
AEC_HIP_LIB=$R/acoustic-echo-cancellation_amd/aec_amd/ab/tick.so timeout -k 10 120 python $R/tools/tick_prof.py > $O/r05f_nlms_tick.txt 2>&1 || { echo "tick prof failed"; tail $O/r05f_nlms_tick.txt; exit 1; }
head -14 $O/r05f_nlms_tick.txt
AEC_FUSED_MODE=32768 AEC_HIP_LIB=$R/acoustic-echo-cancellation_amd/aec_amd/ab/tick.so timeout -k 10 120 python $R/tools/gru_tick_prof.py > $O/r05f_gru_tick_ola.txt 2>&1 || { echo "gru tick prof failed"; tail $O/r05f_gru_tick_ola.txt; exit 1; }
head -14 $O/r05f_gru_tick_ola.txt
