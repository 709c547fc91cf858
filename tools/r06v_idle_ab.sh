#!/bin/bash
# Round 6: the pipelined NS = 1 GRU + synthesis kernel with a 12th, idle wave so the recurrence
# wave's SIMD carries fewer busy waves (AEC_GRU_IDLE = 1..4: four placements; 0: the product's
# 11-wave placement), A/B build; batch 1 / 64 latency alternating, then tick profiles.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/idle; mkdir -p $O
cd $R
export AEC_BENCH_AB=1
for i in 1 2; do
  for m in 0 1 2 3 4; do
    AEC_HIP_LIB=$R/ab_libs/idle.so AEC_GRU_IDLE=$m timeout -k 10 120 python tools/b1_probe.py --sizes 1,64 --reps 20 \
        > $O/m${m}_$i.log 2>&1 || { tail -20 $O/m${m}_$i.log; exit 1; }
    echo "idle $m #$i: $(python -c "
import json
for l in open('$O/m${m}_$i.log'):
    if l.startswith('{'):
        d = json.loads(l); print('B', d['B'], d['ms_median'], d['out_sum'], end='; ')
")"
  done
done
for m in 0 1 2 3 4; do
  echo "== tick profile idle $m"
  AEC_HIP_LIB=$R/ab_libs/tick.so AEC_GRU_IDLE=$m timeout -k 10 100 python tools/gru_tick_prof.py --streams 1 | grep -v 'first stamps' || exit 1
done
