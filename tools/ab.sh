#!/bin/bash
# A/B timing of alternative builds of libaec_hip.so (AEC_HIP_LIB), both pipelines.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/ab
for lib in "$@"; do
  for pl in full postfilter; do
    AEC_HIP_LIB=$R/acoustic-echo-cancellation_amd/aec_amd/ab/$lib.so timeout -k 10 120 python $R/bench.py --no-cpu --no-c3 --no-rtf --steps 20 --pipeline $pl > $R/gpurun_out/ab/$lib.$pl.log 2>&1 || exit 1
    echo "$lib $pl: $(tail -1 $R/gpurun_out/ab/$lib.$pl.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
  done
done
