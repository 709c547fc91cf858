#!/bin/bash
# round 5 batch g: OLA on the gi waves (unrolled), direct frame loads in K2n (ab/direct.so):
# tests, bit-identity across builds, C2 A/B, tick profiles
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
AB=$R/acoustic-echo-cancellation_amd/aec_amd/ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_nlms.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_stream.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r05g_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $O/r05g_tests.log | head -20; tail -5 $O/r05g_tests.log; exit 1; }
tail -1 $O/r05g_tests.log
for lib in tree direct prev; do
  if [ $lib = tree ]; then unset AEC_HIP_LIB; else export AEC_HIP_LIB=$AB/$lib.so; fi
  timeout -k 10 120 python $R/tools/lib_bitcmp.py >> $O/r05g_bitcmp.log 2>&1 || { echo "bitcmp $lib failed"; tail $O/r05g_bitcmp.log; exit 1; }
done
unset AEC_HIP_LIB
grep sha1 $O/r05g_bitcmp.log
bash $R/tools/libs_ab.sh 3 tree acoustic-echo-cancellation_amd/aec_amd/ab/direct.so acoustic-echo-cancellation_amd/aec_amd/ab/prev.so > $O/r05g_ab.log 2>&1 || { echo "ab failed"; tail $O/r05g_ab.log; exit 1; }
cat $O/r05g_ab.log
AEC_HIP_LIB=$AB/tick.so timeout -k 10 120 python $R/tools/gru_tick_prof.py > $O/r05g_gru_tick.txt 2>&1 || { echo "gru tick prof failed"; tail $O/r05g_gru_tick.txt; exit 1; }
head -14 $O/r05g_gru_tick.txt
AEC_HIP_LIB=$AB/tickd.so timeout -k 10 120 python $R/tools/tick_prof.py > $O/r05g_nlms_tick_direct.txt 2>&1 || { echo "tick prof failed"; tail $O/r05g_nlms_tick_direct.txt; exit 1; }
head -14 $O/r05g_nlms_tick_direct.txt
