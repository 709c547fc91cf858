#!/bin/bash
# C2 bench line per batches-in-flight count, alternating rounds: bash tools/inflight_ab.sh "2 3 4" [rounds]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
VALS=${1:-"2 3"}; ROUNDS=${2:-2}
mkdir -p $R/gpurun_out/inflight_ab
for r in $(seq 1 $ROUNDS); do
  for v in $VALS; do
    timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 40 --inflight $v > $R/gpurun_out/inflight_ab/if_${v}_$r.log 2>&1 || exit 1
    echo "round $r inflight=$v: $(tail -1 $R/gpurun_out/inflight_ab/if_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
