#!/bin/bash
# round 5 batch s: look-ahead (moments_lds, 4-round ring) with the compute kernels' waves at
# priority 1 (the co-resident moments waves then take leftover issue slots)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for i in 1 2 3; do for v in "0 0 0 0" "1 3 0 0" "1 3 111 168"; do
  set -- $v
  AEC_MOM_CFG=$2 AEC_NLMS_PRIO=$3 AEC_FUSED_MODE=$4 timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 40 --lookahead $1 > $O/r05s_$1_$2_$3_$4_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05s_$1_$2_$3_$4_$i.log; exit 1; }
  echo "lookahead $1 mom $2 prio $3 fmode $4 #$i: $(tail -1 $O/r05s_$1_$2_$3_$4_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done; done
