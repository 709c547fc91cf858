#!/bin/bash
# rocprofv3 evidence for bench.py on the GPU box (run via gpurun):
#   bash tools/profile.sh <tag> [extra bench args]
# 1. --kernel-trace --stats of the default bench workload (no batch-1 probe, so
#    every traced launch is the bench's 256-stream step);
# 2. FETCH_SIZE and WRITE_SIZE, each in its own --pmc pass (no tracing domains).
# Outputs under gpurun_out/prof_<tag>/; tools/summarize_profile.py turns them
# into profiles/<tag>_* on the build host.
set -euo pipefail
TAG=${1:-r01}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
rm -rf "$OUT"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu --no-c3 --no-train --no-rtf --no-sweep --no-near-leg "$@" > "$OUT/trace_bench.log" 2>&1
echo "trace done"
i=0
for set in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc_$i" -o run -- \
        python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-c3 --no-train --no-rtf --no-sweep --no-near-leg "$@" > "$OUT/pmc_$i.log" 2>&1
    echo "pmc $i done: $set"
done
