#!/bin/bash
# round 5: per-batch completion times inside a 20-step timed region (tools/c2_step_events.py)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for f in 2 3; do
  timeout -k 10 150 python $R/tools/c2_step_events.py --steps 20 --warmup 5 --inflight $f 2>/dev/null | grep '^{' || exit 1
done
timeout -k 10 150 python $R/tools/c2_step_events.py --steps 60 --warmup 5 --inflight 2 2>/dev/null | grep '^{' || exit 1
