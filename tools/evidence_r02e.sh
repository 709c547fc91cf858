#!/bin/bash
# Final round-2 evidence: default bench line, DCCRN bf16 / fp8 kernel traces,
# the C5 per-hop step trace and the training probes (run via gpurun).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python $R/bench.py > $R/gpurun_out/bench_r02e_full.log 2>&1 || exit 1
echo "bench done"
bash $R/tools/crn_prof.sh r02e_crn --dtype bf16 || exit 1
bash $R/tools/crn_prof.sh r02e_crn_fp8 --dtype fp8 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r02e_c5 -o run -- \
    python3 $R/tools/c5_probe.py > $R/gpurun_out/prof_r02e_c5.log 2>&1 || exit 1
bash $R/tools/train_prof.sh || exit 1
echo "evidence done"
