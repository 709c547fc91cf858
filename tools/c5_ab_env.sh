#!/bin/bash
# C5 per-hop step time under alternating environment settings (one box):
#   tools/c5_ab_env.sh <rounds> "VAR=a" "VAR=b" ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
for i in $(seq 1 $N); do
  for e in "$@"; do
    out=$(env $e HOPS=300 timeout -k 10 120 python $R/tools/c5_prof.py 2>/dev/null | grep '^{' | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_hop"])') || exit 1
    echo "$e #$i: $out ms/hop"
  done
done
