#!/bin/bash
# PMC passes over the C5 per-hop step (tools/c5_prof.py: 256 streams, HOPS hops,
# no sweep), one counter group per run, then profiles/pmc_latest_c5.json:
#   1. SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE   2. FETCH_SIZE   3. WRITE_SIZE
# usage: bash tools/c5_pmc.sh <tag>
set -euo pipefail
TAG=${1:-c5pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp HOPS=${HOPS:-50}
cd /tmp
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc_$i" -o run -- \
        python3 "$R/tools/c5_prof.py" > "$OUT/pmc_$i.log" 2>&1
    echo "pmc $i done: $set"
done
cd "$R"
python3 tools/crn_pmc_summary.py "$OUT" "$OUT/summary.json" > "$OUT/summary.txt"
python3 tools/c5_pmc_latest.py "$OUT/summary.json" "$TAG"
