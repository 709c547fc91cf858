#!/bin/bash
# round 5: the driver's own command (bench.py --gpus 1 --steps 20 --warmup 5), C2 only, per batches
# in flight and look-ahead
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for i in 1 2 3; do for v in "1 1" "2 1" "3 1" "2 0" "3 0"; do
  set -- $v
  timeout -k 10 150 python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3 --no-rtf --no-sweep --no-train --inflight $1 --lookahead $2 > $O/r05z3_$1_$2_$i.log 2>&1 || { echo "bench $v failed"; exit 1; }
  echo "inflight $1 lookahead $2 #$i: $(tail -1 $O/r05z3_$1_$2_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done; done
