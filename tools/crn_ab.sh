#!/bin/bash
# A/B of one CRN env knob: bash tools/crn_ab.sh VAR "v1 v2 ..." -> probe line per value
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
VAR=$1; shift
mkdir -p $R/gpurun_out/crn_ab
for v in $1; do
  env $VAR=$v timeout -k 10 180 python $R/tools/crn_probe.py --skip-golden --iters 3 > $R/gpurun_out/crn_ab/${VAR}_$v.log 2>&1 || exit 1
  echo "$VAR=$v: $(tail -1 $R/gpurun_out/crn_ab/${VAR}_$v.log)"
done
