#!/bin/bash
# GRU kernel timing decomposition (AEC_GRU_MODE: 0 full, 1 recurrence only, 2 helpers only; results invalid unless 0)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/gru_modes
for m in 0 1 2; do
  AEC_GRU_MODE=$m timeout -k 10 120 python $R/bench.py --no-cpu --no-c3 --no-rtf --steps 10 --pipeline postfilter > $R/gpurun_out/gru_modes/m$m.log 2>&1 || exit 1
  echo "gru mode $m: $(tail -1 $R/gpurun_out/gru_modes/m$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_ms_per_step"])')"
done
