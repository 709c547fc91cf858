#!/bin/bash
# round 5 batch q: moments_lds with a 5-round ring (32 VGPRs, 20 KiB: fits beside K2n and the
# 160-VGPR gru_synth) under the look-ahead
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for e in 0 3; do AEC_MOM_CFG=$e timeout -k 10 120 python $R/tools/lib_bitcmp.py 2>&1 | grep sha1 >> $O/r05q_bitcmp.log || { echo "bitcmp failed"; exit 1; }; done
cat $O/r05q_bitcmp.log
for i in 1 2 3; do for v in "0 0" "1 3" "0 9"; do
  set -- $v
  AEC_MOM_CFG=$2 timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 40 --lookahead $1 > $O/r05q_la$1_m$2_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05q_la$1_m$2_$i.log; exit 1; }
  echo "lookahead $1 mom $2 #$i: $(tail -1 $O/r05q_la$1_m$2_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
done; done
for i in 1 2; do for d in 1 2; do AEC_MOM_CFG=3 timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 40 --lookahead $d > $O/r05q_d${d}_$i.log 2>&1 || { echo "bench d=$d failed"; tail -5 $O/r05q_d${d}_$i.log; exit 1; }; echo "lookahead $d mom 3 #$i: $(tail -1 $O/r05q_d${d}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"; done; done
