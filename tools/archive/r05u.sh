#!/bin/bash
# round 5 batch u: round-4 final tree (old_r04/: its library, bench.py and defaults -- two batches in
# flight, no look-ahead) against HEAD on one box, C2 only, 100 and 20 timed steps
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for i in 1 2 3; do for k in 100 20; do for t in r04 r05; do
  if [ $t = r04 ]; then B=$R/old_r04/bench.py; else B=$R/bench.py; fi
  timeout -k 10 150 python $B --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps $k > $O/r05u_${t}_${k}_$i.log 2>&1 || { echo "bench $t $k failed"; tail -5 $O/r05u_${t}_${k}_$i.log; exit 1; }
  echo "$t steps $k #$i: $(tail -1 $O/r05u_${t}_${k}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
done; done; done
