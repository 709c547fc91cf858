#!/bin/bash
# Round 6: C2 step, the tree before the small-batch changes (9b47da6) against HEAD, both as A/B builds,
# alternating on one box (the driver's 20-step form and 100 steps).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c2_ab; mkdir -p $O
export AEC_BENCH_AB=1
for i in 1 2 3; do
  for v in pre_ns head_ab; do
    for st in 20 100; do
      AEC_HIP_LIB=$R/ab_libs/$v.so timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-train --no-sweep \
          --steps $st --warmup 5 > $O/${v}_${st}_$i.log 2>&1 || { tail -20 $O/${v}_${st}_$i.log; exit 1; }
      echo "$v steps $st #$i: $(grep '^{' $O/${v}_${st}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("kernel_ms_per_step"))')"
    done
  done
done
