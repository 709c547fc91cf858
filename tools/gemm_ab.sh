#!/bin/bash
# A/B of the row-GEMM cores on the LSTM input-projection shape (tools/probes/gemm_rows_probe).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=$R/tools/probes/gemm_rows_probe
for rep in 1 2; do
  for v in "CRN_GEMM_PIPE=3" "CRN_GEMM_PIPE=4" "CRN_GEMM_PIPE=3 CRN_GEMM_MODE=1" "CRN_GEMM_PIPE=4 CRN_GEMM_MODE=1"; do
    echo -n "$v: "
    env $v timeout -k 5 60 $P 160256 10 || exit 1
  done
done
