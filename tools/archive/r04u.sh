#!/bin/bash
# C5: MX folds (AEC_CRN_STREAM_FUSE bits 3, 4) against stream count
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for s in 256 512 1024 4096; do
  for f in 7 15 31; do
    out=$(env STREAMS=$s AEC_CRN_STREAM_FUSE=$f HOPS=200 timeout -k 10 150 python $R/tools/c5_prof.py 2>/dev/null | grep '^{' | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_hop"], d["frames_per_s_per_gpu"])') || exit 1
    echo "streams=$s FUSE=$f: $out"
  done
done
