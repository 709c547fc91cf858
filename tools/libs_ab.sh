#!/bin/bash
# Alternating A/B of several builds of libaec_hip.so on one box (C2 bench line, no CPU / C3 /
# training / sweep legs).  "tree" = the in-tree library.
#   tools/libs_ab.sh <rounds> tree build_ab/a.so build_ab/b.so ...   [PIPE=full|postfilter|crn]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
PIPE=${PIPE:-full}
O=$R/gpurun_out/libs_ab; mkdir -p $O
for i in $(seq 1 $N); do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    if [ "$lib" = tree ]; then unset AEC_HIP_LIB; else export AEC_HIP_LIB=$R/$lib; fi
    timeout -k 10 150 python $R/bench.py --pipeline $PIPE --no-cpu --no-c3 --no-rtf --no-train --no-sweep --steps 40 \
        > $O/${tag}_$i.log 2>&1 || { tail -20 $O/${tag}_$i.log; exit 1; }
    echo "$tag #$i: $(grep '^{' $O/${tag}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("kernel_ms_per_step") or d.get("stage_ms_per_step"))')"
  done
done
