#!/bin/bash
# A/B of an alternative build of libaec_hip.so (AEC_HIP_LIB) against the in-tree one.
# usage: tools/lib_ab.sh <alt.so> [pipeline]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
ALT=$1; PIPE=${2:-full}
mkdir -p $R/gpurun_out
for v in base alt base alt; do
  if [ $v = alt ]; then export AEC_HIP_LIB=$ALT; else unset AEC_HIP_LIB; fi
  timeout -k 10 120 python $R/bench.py --pipeline $PIPE --no-cpu --no-c3 --no-rtf --steps 50 > $R/gpurun_out/lib_ab_${PIPE}_$v.log 2>&1 || exit 1
  python - "$v" "$R/gpurun_out/lib_ab_${PIPE}_$v.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], 'ms/step', d['ms_per_step'], d.get('kernel_ms_per_step') or d.get('stage_ms_per_step'))
PY
done
