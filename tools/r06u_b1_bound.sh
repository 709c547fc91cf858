#!/bin/bash
# Batch-1 latency bound of a head/synthesis split (A/B library, AEC_FUSED_MODE timing bits; results
# invalid except for 0): 0 all roles; 1031 = synthesis, overlap-add, E loads and head skipped (the
# recurrence + gi + producer floor); 512 = recurrence skipped (the helper roles' own floor).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for i in 1 2; do
  for m in 0 1031 512 1024 7; do
    AEC_HIP_LIB=$R/ab_libs/ab_tree.so AEC_FUSED_MODE=$m timeout -k 10 120 \
        python tools/b1_probe.py --sizes 1,64 --reps 15 >> $O/r06u_b1_bound.log 2>&1 || { tail -20 $O/r06u_b1_bound.log; exit 1; }
  done
done
python - $O/r06u_b1_bound.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print(d['env'].get('AEC_FUSED_MODE'), 'B', d['B'], d['ms_median'], 'ms')
PY
