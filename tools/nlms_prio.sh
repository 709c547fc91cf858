#!/bin/bash
# NLMS analysis kernel time per wave-priority assignment (AEC_NLMS_PRIO = mic|ref|nlms digits).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/nlms_prio
for pr in "$@"; do
  AEC_NLMS_PRIO=$pr timeout -k 10 120 python $R/bench.py --no-cpu --no-c3 --no-rtf --steps 20 > $R/gpurun_out/nlms_prio/p$pr.log 2>&1 || exit 1
  echo "prio $pr: $(tail -1 $R/gpurun_out/nlms_prio/p$pr.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_ms_per_step"]["analysis"], d["ms_per_step"])')"
done
