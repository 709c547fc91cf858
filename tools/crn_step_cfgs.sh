#!/bin/bash
# CRN batch time per LSTM step configuration (CRN_STEP_CFG), 256 x 10 s, bf16
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/step_cfgs
for c in "$@"; do
  CRN_STEP_CFG=$c timeout -k 10 180 python $R/tools/crn_probe.py --skip-golden --iters 3 > $R/gpurun_out/step_cfgs/c$c.log 2>&1 || exit 1
  echo "cfg $c: $(tail -1 $R/gpurun_out/step_cfgs/c$c.log)"
done
