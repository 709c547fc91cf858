#!/bin/bash
# Epilogue decomposition of the LSTM-shape row GEMM: full, no global stores, no epilogue.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for m in 0 2 1; do echo -n "CRN_GEMM_MODE=$m: "; CRN_GEMM_MODE=$m timeout -k 5 60 $R/tools/probes/gemm_rows_probe 160256 10 || exit 1; done
