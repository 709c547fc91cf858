#!/bin/bash
# Round-6 profiles of the final tree (run via gpurun): the C2 bench under rocprofv3 --kernel-trace
# --stats plus the FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh), and the SQ issue / wait
# passes (tools/sq_pmc.sh).  tools/summarize_profile.py and tools/sq_summary.py turn them into
# profiles/ on the build host.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06z}
bash $R/tools/profile.sh ${TAG}_full --inflight 1 || exit 1
bash $R/tools/sq_pmc.sh ${TAG}_sq --inflight 1 || exit 1
echo "evidence done"
