#!/bin/bash
# rocprofv3 kernel trace of the DCCRN probe (config 3 shape): bash tools/crn_prof.sh <tag> [probe args]
set -euo pipefail
TAG=${1:-crn}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/tools/crn_probe.py" --skip-golden --iters 1 "$@" > "$OUT/probe.log" 2>&1
echo "trace done"
