#!/bin/bash
# C5 split-K cap A/B (AEC_CRN_SPLITK: max K slices of the per-hop MX conv GEMMs)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/c5_ab_env.sh 2 AEC_CRN_SPLITK=4 AEC_CRN_SPLITK=8 AEC_CRN_SPLITK=2 || exit 1
