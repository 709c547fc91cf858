#!/bin/bash
# SQ issue / wait counters of the bench kernels (run via gpurun):
#   bash tools/sq_pmc.sh <tag> [extra bench args]
# Two --pmc passes (<= 8 SQ + 1 GRBM counters each, no tracing domains):
#   1. wave / busy / VALU / LDS issue and wait cycles
#   2. LDS bank conflicts, SALU and any-instruction activity
# SQ_*_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* count quad-cycles (MI355X_MICROARCH.md).
# tools/sq_summary.py prints per-kernel ratios.
set -euo pipefail
TAG=${1:-sq}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc_$i" -o run -- \
        python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-c3 --no-rtf --no-train --no-sweep --no-near-leg "$@" > "$OUT/pmc_$i.log" 2>&1
    echo "pmc $i done"
done
