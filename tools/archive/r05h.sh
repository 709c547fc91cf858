#!/bin/bash
# round 5 batch h: the mic_erb pass merged into the mic waves' near ERB (AEC_NLMS_ERB=3) against the
# ref waves' merged pass (1): tests, bit identity, C2 A/B, tick profile
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
AB=$R/acoustic-echo-cancellation_amd/aec_amd/ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_nlms.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_stream.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r05h_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $O/r05h_tests.log | head -20; tail -5 $O/r05h_tests.log; exit 1; }
tail -1 $O/r05h_tests.log
for e in 1 3; do AEC_NLMS_ERB=$e timeout -k 10 120 python $R/tools/lib_bitcmp.py >> $O/r05h_bitcmp.log 2>&1 || { echo "bitcmp failed"; exit 1; }; done
grep sha1 $O/r05h_bitcmp.log
bash $R/tools/env_ab.sh AEC_NLMS_ERB "1 3" 3 > $O/r05h_erb3.log 2>&1 || { echo "ab failed"; tail $O/r05h_erb3.log; exit 1; }
cat $O/r05h_erb3.log
AEC_NLMS_ERB=3 AEC_HIP_LIB=$AB/tick.so timeout -k 10 120 python $R/tools/tick_prof.py > $O/r05h_nlms_tick_erb3.txt 2>&1 || { echo "tick prof failed"; tail $O/r05h_nlms_tick_erb3.txt; exit 1; }
head -14 $O/r05h_nlms_tick_erb3.txt
