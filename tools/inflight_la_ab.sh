#!/bin/bash
# C2 line at 100 timed steps (warm-up floor) for batches in flight x normaliser look-ahead distance,
# alternating rounds on one box.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/inflight_la
mkdir -p $O
B="--no-cpu --no-c3 --no-rtf --no-sweep --no-train"
for r in 1 2; do
  for cfg in 3:1 4:1 3:0 4:2; do
    IFS=: read inf la <<< "$cfg"
    timeout -k 10 200 python $R/bench.py $B --inflight $inf --lookahead $la > $O/i${inf}_la${la}_$r.log 2>&1 \
        || { echo "bench failed"; tail -20 $O/i${inf}_la${la}_$r.log; exit 1; }
    echo "round $r inflight=$inf lookahead=$la: $(tail -1 $O/i${inf}_la${la}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
bash $R/tools/cumask_ab.sh
