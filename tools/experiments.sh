#!/bin/bash
# Ad-hoc timing experiments on the GPU box (run via gpurun).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/exp
mkdir -p "$OUT"
for m in 0 1 2; do
  AEC_GRU_MODE=$m timeout -k 10 200 python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-c3 > "$OUT/gru_mode_$m.json" 2>"$OUT/gru_mode_$m.err" || exit 1
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES \
   --output-format csv -d "$OUT/pmc_lds" -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-c3 > "$OUT/pmc_lds.log" 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
   --output-format csv -d "$OUT/pmc_wait" -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-c3 > "$OUT/pmc_wait.log" 2>&1
echo done
