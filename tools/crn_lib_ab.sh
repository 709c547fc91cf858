#!/bin/bash
# C3 stage A/B of an alternative libaec_hip.so (AEC_HIP_LIB) against the in-tree one, alternating.
# usage: tools/crn_lib_ab.sh <alt.so> [extra bench args]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
ALT=$1; shift
mkdir -p $R/gpurun_out
for v in base alt base alt; do
  if [ $v = alt ]; then export AEC_HIP_LIB=$ALT; else unset AEC_HIP_LIB; fi
  timeout -k 10 200 python $R/bench.py --pipeline crn --steps 5 --warmup 2 --no-cpu --no-rtf --no-sweep --crn-inflight 1 "$@" > $R/gpurun_out/crn_lib_ab_$v.log 2>&1 || { tail -5 $R/gpurun_out/crn_lib_ab_$v.log; exit 1; }
  python - "$v" "$R/gpurun_out/crn_lib_ab_$v.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], 'ms/step', d['ms_per_step'], d.get('stage_ms_per_step'))
PY
done
