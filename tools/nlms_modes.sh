#!/bin/bash
# Timing decomposition of the NLMS analysis kernel (AEC_NLMS_MODE bits; results invalid unless 0).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/nlms_modes
for m in 0 1 2 4 8 7 9 15; do
  AEC_NLMS_MODE=$m timeout -k 10 120 python $R/bench.py --no-cpu --no-c3 --no-rtf --steps 10 > $R/gpurun_out/nlms_modes/m$m.log 2>&1 || exit 1
  echo "mode $m: $(tail -1 $R/gpurun_out/nlms_modes/m$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_ms_per_step"])')"
done
