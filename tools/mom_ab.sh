#!/bin/bash
# A/B of the moments kernel variants (AEC_MOM_CFG) on the default bench.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for c in ${CFGS:-0 1 2 3 4 5 0}; do
  AEC_MOM_CFG=$c timeout -k 10 120 python $R/bench.py --no-cpu --no-c3 --no-rtf --steps 50 > $R/gpurun_out/mom_ab_$c.log 2>&1 || exit 1
  python - "$c" "$R/gpurun_out/mom_ab_$c.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print('cfg', sys.argv[1], 'ms/step', d['ms_per_step'], d['kernel_ms_per_step'])
PY
done
