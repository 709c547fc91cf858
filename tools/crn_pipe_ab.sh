#!/bin/bash
# C3 (DCCRN bf16, 256 x 10 s) bench line per CRN_GEMM_PIPE setting (row-GEMM cores).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for p in 0 2 3; do
  echo "CRN_GEMM_PIPE=$p"
  CRN_GEMM_PIPE=$p timeout -k 10 150 python $R/bench.py --pipeline crn --steps 10 --no-cpu --no-rtf > $R/gpurun_out/crn_pipe_$p.json || exit 1
  python -c "import json,sys; d=json.loads(open('$R/gpurun_out/crn_pipe_$p.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('stage_ms_per_step'))"
done
