#!/bin/bash
# full-pipeline step time vs batch size, split NLMS path (AEC_SMALLB=100000) against K2n (AEC_SMALLB=0)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/smallb
for b in "$@"; do
  for sb in 0 100000; do
    AEC_SMALLB=$sb timeout -k 10 120 python $R/bench.py --no-cpu --no-c3 --no-rtf --streams $b --steps 20 > $R/gpurun_out/smallb/b${b}_s$sb.log 2>&1 || exit 1
    echo "B $b smallb $sb: $(tail -1 $R/gpurun_out/smallb/b${b}_s$sb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_ms_per_step"], d["ms_per_step"])')"
  done
done
