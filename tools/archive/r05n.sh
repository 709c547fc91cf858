#!/bin/bash
# round 5 batch n: the normaliser look-ahead with a persistent moments pass (AEC_MOM_CFG=4,
# AEC_MOM_GRID blocks) that shares CUs with the analysis kernel; cfg 9 = no pass (timing floor)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for e in 0 4; do AEC_MOM_CFG=$e timeout -k 10 120 python $R/tools/lib_bitcmp.py 2>&1 | grep sha1 >> $O/r05n_bitcmp.log || { echo "bitcmp failed"; exit 1; }; done
cat $O/r05n_bitcmp.log
for i in 1 2; do for v in "0 256" "3 256" "4 256" "4 128" "4 64" "9 256"; do
  set -- $v
  AEC_MOM_CFG=$1 AEC_MOM_GRID=$2 timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 40 > $O/r05n_m$1_g$2_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05n_m$1_g$2_$i.log; exit 1; }
  echo "mom $1 grid $2 #$i: $(tail -1 $O/r05n_m$1_g$2_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
done; done
