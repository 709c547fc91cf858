#!/bin/bash
# C2 line at 100 timed steps with the look-ahead side stream CU-masked (bench.py --lookahead-cus N),
# alternating rounds on one box; N = 0 is the unmasked default.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/cumask
mkdir -p $O
B="--no-cpu --no-c3 --no-rtf --no-sweep --no-train"
for r in 1 2 3; do
  for n in 0 32 64 16 128; do
    timeout -k 10 200 python $R/bench.py $B --lookahead-cus $n > $O/cus${n}_$r.log 2>&1 \
        || { echo "bench failed"; tail -20 $O/cus${n}_$r.log; exit 1; }
    echo "round $r lookahead_cus=$n: $(tail -1 $O/cus${n}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
