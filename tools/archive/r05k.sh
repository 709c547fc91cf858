#!/bin/bash
# round 5 batch k: the C2 step without the moments pass (timing-only upper bound for hiding it)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
bash $R/tools/env_ab.sh AEC_MOM_CFG "0 3 9" 3 > $O/r05k_mom.log 2>&1 || { echo "ab failed"; tail $O/r05k_mom.log; exit 1; }
cat $O/r05k_mom.log
