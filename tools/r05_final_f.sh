#!/bin/bash
# round-5 end-of-round evidence (6/6): the driver's own command line, twice, and the default line
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for i in 1 2; do
  timeout -k 10 500 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/r05zg_driver_$i.log 2>&1 || { echo "bench failed"; tail -20 $O/r05zg_driver_$i.log; exit 1; }
  tail -1 $O/r05zg_driver_$i.log | head -c 420; echo
done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05zg_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/r05zg_smoke.log
