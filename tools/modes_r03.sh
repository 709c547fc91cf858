#!/bin/bash
# Timing decomposition of the two headline kernels (timing-only env bits; results invalid unless 0):
#   AEC_NLMS_MODE  (nlms_analysis_kernel): 1 no recursion, 2 no near ERB, 4 no mic_erb pass, 8 no transforms
#   AEC_FUSED_MODE (gru_synth_kernel): 1 no synthesis, 2 no OLA, 4 no E loads, 512 no recurrence, 1024 no head, 2048 no gi
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/modes_r03; mkdir -p $O
run() {  # var value
  env $1=$2 timeout -k 10 120 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-train --no-sweep --steps 10 > $O/$1_$2.log 2>&1 || exit 1
  echo "$1=$2: $(grep '^{' $O/$1_$2.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_ms_per_step"], d["ms_per_step"])')"
}
for m in ${NLMS_MODES:-}; do run AEC_NLMS_MODE $m; done
for m in ${FUSED_MODES:-}; do run AEC_FUSED_MODE $m; done
