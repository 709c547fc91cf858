#!/bin/bash
# round 5 batch x: C5 per-hop step with and without the hipGraph (AEC_CRN_GRAPH): the 8.2-us gap
# between consecutive graph launches against per-kernel launch gaps
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/c5_ab_env.sh 3 "AEC_CRN_GRAPH=1" "AEC_CRN_GRAPH=0"
