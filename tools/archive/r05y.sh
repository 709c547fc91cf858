#!/bin/bash
# round 5 batch y: C5 with / without the hipGraph at 256 and 4,096 streams and one stream
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for i in 1 2; do for s in 256 4096; do for g in 1 0; do
  out=$(AEC_CRN_GRAPH=$g STREAMS=$s HOPS=200 timeout -k 10 150 python $R/tools/c5_prof.py 2>/dev/null | grep '^{' | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_hop"], json.dumps(d.get("batch1")))') || exit 1
  echo "streams $s graph $g #$i: $out"
done; done; done
