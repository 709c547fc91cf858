#!/bin/bash
# C5 fused LSTM launch vs two launches per stream count (is the 2-blocks-per-CU residency reached?)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for B in 32 64 128 192 256; do
  for f in 1 0; do
    AEC_CRN_LSTM_FUSE=$f STREAMS=$B HOPS=300 timeout -k 10 120 python tools/c5_mode_prof.py >> $O/r06y_streams.log 2>&1 \
        || { tail -20 $O/r06y_streams.log; exit 1; }
    echo "B=$B fuse=$f $(tail -1 $O/r06y_streams.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_hop"], d["stats"]["lstm_launches_per_hop"])')"
  done
done
