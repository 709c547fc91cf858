#!/bin/bash
# L2 hit rate of the DCCRN kernels: one --pmc pass (TCC_HIT_sum, TCC_MISS_sum) over the probe
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_crnl2
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc" -o run -- \
    python3 "$R/tools/crn_probe.py" --skip-golden --iters 1 --B 256 --N 32000 "$@" > "$OUT/probe.log" 2>&1
echo "pmc done"
