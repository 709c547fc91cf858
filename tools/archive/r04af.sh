#!/bin/bash
# PMC refresh on the final build: C5 per-hop step (MFMA busy, FETCH, WRITE) and C3 bf16 (same groups)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
bash $R/tools/c5_pmc.sh r04zz_c5pmc > $R/gpurun_out/r04af_c5.log 2>&1 || { echo "c5 pmc failed"; tail -5 $R/gpurun_out/r04af_c5.log; exit 1; }
echo "c5 pmc done"
bash $R/tools/crn_pmc.sh r04zz_crnpmc > $R/gpurun_out/r04af_crn.log 2>&1 || { echo "crn pmc failed"; tail -5 $R/gpurun_out/r04af_crn.log; exit 1; }
echo "crn pmc done"
