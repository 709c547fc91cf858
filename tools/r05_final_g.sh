#!/bin/bash
# round-5 end-of-round evidence (7): the GPU suite, smoke and the default bench line on the final tree
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/r05zl_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/r05zl_gputest.log; exit 1; }
tail -1 $O/r05zl_gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05zl_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/r05zl_smoke.log
timeout -k 10 600 python3 $R/bench.py > $O/r05zl_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/r05zl_bench.log; exit 1; }
tail -1 $O/r05zl_bench.log | head -c 600; echo
