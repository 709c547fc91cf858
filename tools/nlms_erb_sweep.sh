#!/bin/bash
# NLMS analysis time per (mic_erb role, wave priorities): args "erb:prio" pairs
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/nlms_erb
for ep in "$@"; do
  e=${ep%%:*}; pr=${ep##*:}
  AEC_NLMS_ERB=$e AEC_NLMS_PRIO=$pr timeout -k 10 120 python $R/bench.py --no-cpu --no-c3 --no-rtf --steps 20 > $R/gpurun_out/nlms_erb/e${e}_p$pr.log 2>&1 || exit 1
  echo "erb $e prio $pr: $(tail -1 $R/gpurun_out/nlms_erb/e${e}_p$pr.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_ms_per_step"]["analysis"], d["ms_per_step"])')"
done
