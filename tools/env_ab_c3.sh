#!/bin/bash
# C3 (DCCRN bf16 batch, 256 x 10 s) under alternating environment settings on one box; the line
# carries the output's SHA-1 (bit-identity across settings):
#   bash tools/env_ab_c3.sh <rounds> [--dtype fp8] -- "VAR=a" "VAR=b" ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
EXTRA=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do EXTRA+=("$1"); shift; done
shift
mkdir -p $R/gpurun_out/env_ab
for i in $(seq 1 $N); do
  for e in "$@"; do
    env $e timeout -k 10 180 python $R/tools/crn_probe.py --skip-golden --iters 3 "${EXTRA[@]}" > $R/gpurun_out/env_ab/c3_$i.log 2>&1 || { echo "$e failed"; tail -5 $R/gpurun_out/env_ab/c3_$i.log; exit 1; }
    echo "$e #$i: $(tail -1 $R/gpurun_out/env_ab/c3_$i.log)"
  done
done
