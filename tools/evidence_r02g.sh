#!/bin/bash
# Round-2 final evidence (r02g): GPU suite, smoke, default bench line, DCCRN bf16 kernel trace.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02g_gputest.log 2>&1 || exit 1
echo "tests done"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02g_smoke.log 2>&1 || exit 1
echo "smoke done"
timeout -k 10 400 python bench.py > gpurun_out/r02g_bench_final.log 2>&1 || exit 1
echo "bench done"
bash tools/crn_prof.sh r02g_crn --dtype bf16 || exit 1
echo "evidence done"
