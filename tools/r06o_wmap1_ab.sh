#!/bin/bash
# Round 6: role-to-SIMD placements of the NS = 1 GRU + synthesis kernel (small batches, pipelined
# split path), A/B build AEC_GRU_WMAP 0..4: batch 1 / 64 latency alternating, then tick profiles.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/wmap1; mkdir -p $O
cd $R
export AEC_BENCH_AB=1
for i in 1 2; do
  for m in 0 1 2 3 4; do
    AEC_HIP_LIB=$R/ab_libs/wmap.so AEC_GRU_WMAP=$m timeout -k 10 120 python tools/b1_probe.py --sizes 1,64,128 --reps 20 \
        > $O/m${m}_$i.log 2>&1 || { tail -20 $O/m${m}_$i.log; exit 1; }
    echo "wmap $m #$i: $(python -c "
import json
for l in open('$O/m${m}_$i.log'):
    if l.startswith('{'):
        d = json.loads(l); print('B', d['B'], d['ms_median'], d['out_sum'], end='; ')
")"
  done
done
for m in 0 1 2 3 4; do
  echo "== tick profile wmap $m"
  AEC_HIP_LIB=$R/ab_libs/tick.so AEC_GRU_WMAP=$m timeout -k 10 100 python tools/gru_tick_prof.py --streams 1 | grep -v 'first stamps' || exit 1
done
