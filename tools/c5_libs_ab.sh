#!/bin/bash
# Alternating A/B of the C5 per-hop step (256 streams, fp8, hipGraph) over library builds / env settings:
#   tools/c5_libs_ab.sh <rounds> "tag|lib|ENV=V ..." ...      (lib: a path under the repo, or "tree")
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
O=$R/gpurun_out/c5_libs_ab; mkdir -p $O
for i in $(seq 1 $N); do
  for spec in "$@"; do
    IFS='|' read -r tag lib envs <<< "$spec"
    if [ "$lib" = tree ]; then unset AEC_HIP_LIB; else export AEC_HIP_LIB=$R/$lib; fi
    env $envs timeout -k 10 150 python $R/tools/c5_prof.py > $O/${tag}_$i.log 2>&1 || { tail -20 $O/${tag}_$i.log; exit 1; }
    echo "$tag #$i: $(tail -1 $O/${tag}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_hop"])')"
  done
done
