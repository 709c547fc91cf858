#!/bin/bash
# rocprofv3 kernel trace of the C5 per-hop step: bash tools/c5_prof.sh <tag>
set -euo pipefail
TAG=${1:-c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/tools/c5_prof.py" > "$OUT/c5.log" 2>&1
echo "c5 trace done"
