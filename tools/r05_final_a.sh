#!/bin/bash
# round-5 end-of-round evidence (1/3): GPU suite (parity margins), smoke, default bench line
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/r05z_gputest.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error" $O/r05z_gputest.log | head; tail -30 $O/r05z_gputest.log; exit 1; }
tail -1 $O/r05z_gputest.log
cp $O/parity_margins.json $O/r05z_parity_margins.json
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05z_smoke.log 2>&1 || { echo "smoke failed"; tail $O/r05z_smoke.log; exit 1; }
tail -1 $O/r05z_smoke.log
timeout -k 10 500 python $R/bench.py > $O/r05z_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/r05z_bench.log; exit 1; }
tail -1 $O/r05z_bench.log | head -c 600; echo
