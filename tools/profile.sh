#!/bin/bash
# Kernel-trace + PMC profile of bench.py on the GPU box (run via gpurun).
#   bash tools/profile.sh <tag> [extra bench args]
# Writes gpurun_out/prof_<tag>/{trace,pmc_*}/... ; summaries are copied into
# profiles/ by tools/summarize_profile.py afterwards (on the build host).
set -euo pipefail
TAG=${1:-r01}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --steps 10 --warmup 2 --no-cpu $*"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $B \
    > "$OUT/trace_bench.log" 2>&1
echo "trace done"
# PMC passes (each in its own run; no tracing domains combined with --pmc)
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc_$i" -o run -- python3 $R/bench.py \
        --steps 2 --warmup 1 --no-cpu $* > "$OUT/pmc_$i.log" 2>&1
    echo "pmc $i done: $set"
done
