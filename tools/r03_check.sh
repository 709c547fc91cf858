#!/bin/bash
# Round 3 check: GPU suite (verbose, per-test timeout), smoke, default bench line.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03a}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 150 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -60 gpurun_out/${TAG}_gputest.log; exit 1; }
echo "tests done"; tail -3 gpurun_out/${TAG}_gputest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
echo "smoke done"
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
echo "bench done"
