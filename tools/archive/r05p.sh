#!/bin/bash
# round 5 batch p: gru_synth at 160 VGPRs (overlap-add on the recurrence waves at compile time) so
# a 30-VGPR moments_lds wave fits beside both compute kernels; look-ahead A/B with cfg 0 / 3
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_nlms.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r05p_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $O/r05p_tests.log | head -20; tail -5 $O/r05p_tests.log; exit 1; }
tail -1 $O/r05p_tests.log
for e in 0 3; do AEC_MOM_CFG=$e timeout -k 10 120 python $R/tools/lib_bitcmp.py 2>&1 | grep sha1 >> $O/r05p_bitcmp.log || { echo "bitcmp failed"; exit 1; }; done
cat $O/r05p_bitcmp.log
for i in 1 2 3; do for v in "0 0" "0 3" "1 0" "1 3"; do
  set -- $v
  AEC_MOM_CFG=$2 timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 40 --lookahead $1 > $O/r05p_la$1_m$2_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05p_la$1_m$2_$i.log; exit 1; }
  echo "lookahead $1 mom $2 #$i: $(tail -1 $O/r05p_la$1_m$2_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
done; done
