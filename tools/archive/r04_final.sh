#!/bin/bash
# round-4 end-of-session evidence: GPU suite, smoke, default bench line, C2 rocprofv3 trace + HBM passes
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 240 --timeout-method thread > $R/gpurun_out/r04z_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $R/gpurun_out/r04z_gputest.log; exit 1; }
tail -1 $R/gpurun_out/r04z_gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/r04z_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $R/gpurun_out/r04z_smoke.log
timeout -k 10 400 python $R/bench.py > $R/gpurun_out/r04z_bench.log 2>&1 || { echo "bench failed"; tail -20 $R/gpurun_out/r04z_bench.log; exit 1; }
echo "bench done"
bash $R/tools/profile.sh r04z_full --inflight 1 || exit 1
echo "profile done"
