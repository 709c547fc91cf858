#!/bin/bash
# round 5 batch i: gru_synth overlap-add on the recurrence waves (AEC_FUSED_MODE bit 15): tests,
# bit identity, C2 A/B, gru tick profile
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
AB=$R/acoustic-echo-cancellation_amd/aec_amd/ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_nlms.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_stream.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r05i_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $O/r05i_tests.log | head -20; tail -5 $O/r05i_tests.log; exit 1; }
tail -1 $O/r05i_tests.log
for e in 0 32768; do AEC_FUSED_MODE=$e timeout -k 10 120 python $R/tools/lib_bitcmp.py >> $O/r05i_bitcmp.log 2>&1 || { echo "bitcmp failed"; exit 1; }; done
grep sha1 $O/r05i_bitcmp.log
bash $R/tools/env_ab.sh AEC_FUSED_MODE "0 32768" 3 > $O/r05i_olarec.log 2>&1 || { echo "ab failed"; tail $O/r05i_olarec.log; exit 1; }
cat $O/r05i_olarec.log
AEC_FUSED_MODE=32768 AEC_HIP_LIB=$AB/tick.so timeout -k 10 120 python $R/tools/gru_tick_prof.py > $O/r05i_gru_tick_olarec.txt 2>&1 || { echo "gru tick failed"; tail $O/r05i_gru_tick_olarec.txt; exit 1; }
head -14 $O/r05i_gru_tick_olarec.txt
