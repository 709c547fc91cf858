#!/bin/bash
# SQ issue / wait counters of the DCCRN kernels (two --pmc passes over a short probe).
# tools/sq_summary.py gpurun_out/prof_crnsq prints per-kernel ratios.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_crnsq
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc_$i" -o run -- \
        python3 "$R/tools/crn_probe.py" --skip-golden --iters 1 --B 256 --N 32000 "$@" > "$OUT/pmc_$i.log" 2>&1
    echo "pmc $i done"
done
