#!/bin/bash
# round 5 batch o: a valid floor for hiding the moments pass (cfg 9 now skips it only after every
# handle's workspace holds real partials; --lookahead 0 so the workspaces are the ones used)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for i in 1 2 3; do for m in 0 9; do
  AEC_MOM_CFG=$m timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 40 --lookahead 0 > $O/r05o_m${m}_$i.log 2>&1 || { echo "bench failed"; tail -5 $O/r05o_m${m}_$i.log; exit 1; }
  echo "mom $m #$i: $(tail -1 $O/r05o_m${m}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"], d.get("erle"))')"
done; done
bash $R/tools/r05p.sh
