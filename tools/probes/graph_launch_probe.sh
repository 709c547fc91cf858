#!/bin/bash
# runs tools/probes/graph_launch_probe in each variant (see its header)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=$R/tools/probes/graph_launch_probe
for v in 0 5; do timeout -k 5 60 $P $v || exit 1; done
