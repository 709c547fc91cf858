#!/bin/bash
# Round evidence on the GPU box: default bench (with cpu_baseline), the
# post-filter-only bench, and rocprofv3 trace + PMC passes for both pipelines.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
mkdir -p $R/gpurun_out
timeout -k 10 300 python $R/bench.py > $R/gpurun_out/bench_${TAG}_full.log 2>&1 || exit 1
echo "bench full done"
timeout -k 10 300 python $R/bench.py --pipeline postfilter > $R/gpurun_out/bench_${TAG}_postfilter.log 2>&1 || exit 1
echo "bench postfilter done"
# traces with one batch in flight: kernel durations without a concurrent batch,
# the configuration of bench.py's own per-kernel timing pass
bash $R/tools/profile.sh ${TAG}_full --pipeline full --inflight 1 || exit 1
bash $R/tools/profile.sh ${TAG}_postfilter --pipeline postfilter --inflight 1 || exit 1
echo "profiles done"
