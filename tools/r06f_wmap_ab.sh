#!/bin/bash
# Round 6: gru_synth role-to-SIMD placements (AEC_GRU_WMAP 0..4, an A/B build) on the C2
# pipeline, then the per-role tick profile of each placement (a -DAEC_TICK_PROF build).
#   bash tools/r06f_wmap_ab.sh <rounds>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-3}
O=$R/gpurun_out/wmap_ab; mkdir -p $O
export AEC_BENCH_AB=1
export AEC_HIP_LIB=$R/ab_libs/wmap.so
for i in $(seq 1 $N); do
  for m in 0 1 2 3 4; do
    AEC_GRU_WMAP=$m timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-train --no-sweep --steps 100 \
        > $O/m${m}_$i.log 2>&1 || { tail -20 $O/m${m}_$i.log; exit 1; }
    echo "wmap $m #$i: $(grep '^{' $O/m${m}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("kernel_ms_per_step"))')"
  done
done
export AEC_HIP_LIB=$R/ab_libs/wmap_tick.so
for m in 0 1 2 3 4; do
  echo "== tick profile wmap $m"
  AEC_GRU_WMAP=$m timeout -k 10 150 python $R/tools/gru_tick_prof.py || exit 1
done
