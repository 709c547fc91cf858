#!/bin/bash
# PMC passes over the DCCRN probe (config 3 shape), one counter group per run:
#   1. SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE (MFMA utilisation)
#   2. FETCH_SIZE   3. WRITE_SIZE   (HBM bytes, MI355X_MICROARCH.md HBM section)
set -euo pipefail
TAG=${1:-crnpmc}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc_$i" -o run -- \
        python3 "$R/tools/crn_probe.py" --skip-golden --iters 1 "$@" > "$OUT/pmc_$i.log" 2>&1
    echo "pmc $i done: $set"
done
