#!/bin/bash
# round 5 batch j: the LDS-DMA moments pass (AEC_MOM_CFG=3: 30 VGPRs, fits beside a K2n block):
# bit identity, C2 A/B with two batches in flight
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for e in 0 3; do AEC_MOM_CFG=$e timeout -k 10 120 python $R/tools/lib_bitcmp.py >> $O/r05j_bitcmp.log 2>&1 || { echo "bitcmp failed"; tail $O/r05j_bitcmp.log; exit 1; }; done
grep sha1 $O/r05j_bitcmp.log
bash $R/tools/env_ab.sh AEC_MOM_CFG "0 3" 4 > $O/r05j_mom.log 2>&1 || { echo "ab failed"; tail $O/r05j_mom.log; exit 1; }
cat $O/r05j_mom.log
