#!/bin/bash
# round 5 batch r: (1) the 8-wave persistent LSTM recurrence (crn_persist3.hip): persistent tests,
# C3 A/B; (2) look-ahead with the 4- / 5-round moments ring against no look-ahead
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
AB=$R/acoustic-echo-cancellation_amd/aec_amd/ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_crn.py -m gpu -x -v -k persistent --timeout 240 --timeout-method thread > $O/r05r_tests.log 2>&1 || { echo "persistent tests failed"; grep -E "PASS|FAIL|Error|assert" $O/r05r_tests.log | head -20; tail -5 $O/r05r_tests.log; exit 1; }
grep -E "PASSED|passed|failed" $O/r05r_tests.log | tail -5
bash $R/tools/env_ab_c3.sh 2 -- "AEC_CRN_PERSIST_WAVES=4" "AEC_CRN_PERSIST_WAVES=8" > $O/r05r_c3.log 2>&1 || { echo "c3 ab failed"; tail $O/r05r_c3.log; exit 1; }
cat $O/r05r_c3.log
for i in 1 2 3 4; do for v in "0 0 tree" "1 3 tree" "1 3 mom5"; do
  set -- $v
  if [ $3 = tree ]; then unset AEC_HIP_LIB; else export AEC_HIP_LIB=$AB/$3.so; fi
  AEC_MOM_CFG=$2 timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 40 --lookahead $1 > $O/r05r_la$1_m$2_$3_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05r_la$1_m$2_$3_$i.log; exit 1; }
  echo "lookahead $1 mom $2 $3 #$i: $(tail -1 $O/r05r_la$1_m$2_$3_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done; done
