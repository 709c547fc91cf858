#!/bin/bash
# Round-2 (session f) evidence, part 2: rocprofv3 kernel trace + HBM passes of the
# headline, DCCRN bf16 kernel trace and PMC passes.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/profile.sh r02f_full --pipeline full --inflight 1 || exit 1
bash tools/crn_prof.sh r02f_crn --dtype bf16 || exit 1
bash tools/crn_pmc.sh r02f_crnpmc --dtype bf16 || exit 1
echo "evidence done"
