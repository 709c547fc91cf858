#!/bin/bash
# Round 6: the canonical moments pass (f32 pre-summed units, one wave per item) against the
# round-5 HEAD library, and its A/B forms (chunk order, cache policy) with and without look-ahead.
#   bash tools/mom_ab.sh <rounds>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-3}
O=$R/gpurun_out/mom_ab; mkdir -p $O
export AEC_BENCH_AB=1
run() {   # tag lib lookahead [env...]
  local tag=$1 lib=$2 la=$3; shift 3
  if [ "$lib" = tree ]; then unset AEC_HIP_LIB; else export AEC_HIP_LIB=$R/$lib; fi
  env "$@" timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-train --no-sweep --steps 100 \
      --lookahead $la > $O/${tag}_$i.log 2>&1 || { tail -20 $O/${tag}_$i.log; exit 1; }
  echo "$tag #$i: $(grep '^{' $O/${tag}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("kernel_ms_per_step"))')"
}
for i in $(seq 1 $N); do
  run base ab_libs/base.so 1
  run canon tree 1
  run canon_la0 tree 0
  run ab_rev_default_la0 ab_libs/mom_ab.so 0 AEC_MOM_ORDER=1 AEC_MOM_AUX=0
  run ab_default_la1 ab_libs/mom_ab.so 1 AEC_MOM_AUX=0
done
