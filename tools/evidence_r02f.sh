#!/bin/bash
# Round-2 (session f) evidence: GPU suite, smoke, default bench line, rocprofv3
# kernel trace + HBM passes of the headline, DCCRN bf16 trace, DCCRN bf16 PMC passes.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02f_gputest.log 2>&1 || exit 1
echo "tests done"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02f_smoke.log 2>&1 || exit 1
echo "smoke done"
timeout -k 10 400 python bench.py > gpurun_out/r02f_bench_full.log 2>&1 || exit 1
echo "bench done"
bash tools/profile.sh r02f_full || exit 1
bash tools/crn_prof.sh r02f_crn --dtype bf16 || exit 1
bash tools/crn_pmc.sh r02f_crnpmc --dtype bf16 || exit 1
echo "evidence done"
