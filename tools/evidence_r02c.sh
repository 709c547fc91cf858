#!/bin/bash
# Round-2 (session c) evidence on the GPU box: default bench (all figures,
# cpu baselines), post-filter bench, rocprofv3 trace + HBM PMC of both AEC
# pipelines (1 batch in flight), DCCRN bf16 / fp8 kernel traces.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/round_evidence.sh r02c || exit 1
bash $R/tools/crn_prof.sh r02c_crn --dtype bf16 || exit 1
bash $R/tools/crn_prof.sh r02c_crn_fp8 --dtype fp8 || exit 1
echo "evidence done"
