#!/bin/bash
# C5 per-hop step: the two MX LSTM layers in one launch (AEC_CRN_LSTM_FUSE=1, default) against two
# launches (0).  1. the bit-exactness tests; 2. ms per hop alternating, direct launches and graph
# replays (tools/c5_mode_prof.py, 400 hops after 60 warm-up hops); 3. kernel traces of both (hop table).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shapes.py -x -v --timeout 300 --timeout-method thread \
    -k "one_launch or graph_replay or 256_streams" > $O/r06x_test.log 2>&1 || { tail -40 $O/r06x_test.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/r06x_test.log | tail -8
for i in 1 2 3; do
  for f in 1 0; do
    for g in 0 1; do
      AEC_CRN_LSTM_FUSE=$f C5_GRAPH=$g HOPS=400 timeout -k 10 120 python tools/c5_mode_prof.py >> $O/r06x_ab.log 2>&1 \
          || { tail -20 $O/r06x_ab.log; exit 1; }
      echo "fuse=$f graph=$g $(tail -1 $O/r06x_ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_hop"], d["stats"]["lstm_launches_per_hop"])')"
    done
  done
done
export TMPDIR=/tmp
for f in 1 0; do
  rm -rf $O/prof_r06x_f$f; mkdir -p $O/prof_r06x_f$f
  (cd /tmp && AEC_CRN_LSTM_FUSE=$f HOPS=200 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/prof_r06x_f$f/trace -o run -- python3 $R/tools/c5_mode_prof.py > $O/prof_r06x_f$f/c5.log 2>&1) \
      || { tail -20 $O/prof_r06x_f$f/c5.log; exit 1; }
done
python tools/c5_hop_table.py $O/prof_r06x_f1 $O/prof_r06x_f0 > $O/r06x_hop_table.txt 2>&1; cat $O/r06x_hop_table.txt
