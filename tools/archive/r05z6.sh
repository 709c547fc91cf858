#!/bin/bash
# round 5: does a longer warm-up remove the slow first batches of a 20-step region?
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for w in 5 40 80; do
  timeout -k 10 150 python $R/tools/c2_step_events.py --steps 20 --warmup $w --inflight 2 --paced 0 2>/dev/null | grep '^{' | cut -c1-600 || exit 1
done
for i in 1 2; do for w in 5 40; do for f in 2 3; do
  timeout -k 10 150 python $R/bench.py --gpus 1 --steps 20 --warmup $w --no-cpu --no-c3 --no-rtf --no-sweep --no-train --inflight $f > /tmp/b.log 2>&1 || { echo "bench failed"; exit 1; }
  echo "warmup $w inflight $f #$i: $(tail -1 /tmp/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done; done; done
