#!/bin/bash
# round 5: the look-ahead passes paced by batch completion (bench.py) at the driver's command
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 150 python $R/tools/c2_step_events.py --steps 20 --warmup 5 --inflight 2 --paced 1 2>/dev/null | grep '^{' | cut -c1-700 || exit 1
for i in 1 2 3; do for f in 2 3; do
  timeout -k 10 150 python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3 --no-rtf --no-sweep --no-train --inflight $f > $O/r05z5_${f}_$i.log 2>&1 || { echo "bench failed"; exit 1; }
  echo "paced inflight $f steps 20 #$i: $(tail -1 $O/r05z5_${f}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done; done
for f in 2 3; do
  timeout -k 10 150 python $R/bench.py --gpus 1 --steps 100 --warmup 5 --no-cpu --no-c3 --no-rtf --no-sweep --no-train --inflight $f > $O/r05z5_100_$f.log 2>&1 || { echo "bench failed"; exit 1; }
  echo "paced inflight $f steps 100: $(tail -1 $O/r05z5_100_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
