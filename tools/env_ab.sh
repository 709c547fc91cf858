#!/bin/bash
# C2 bench line per value of one env knob, alternating rounds:
#   bash tools/env_ab.sh VAR "v1 v2" [rounds] -> ms_per_step and per-kernel ms per run
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
VAR=$1; VALS=$2; ROUNDS=${3:-2}
mkdir -p $R/gpurun_out/env_ab
for r in $(seq 1 $ROUNDS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 20 > $R/gpurun_out/env_ab/${VAR}_${v}_$r.log 2>&1 || exit 1
    echo "round $r $VAR=$v: $(tail -1 $R/gpurun_out/env_ab/${VAR}_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
  done
done
