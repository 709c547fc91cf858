#!/bin/bash
# Fused GRU + synthesis kernel time per AEC_FUSED_MODE (timing only; results invalid unless 0)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/fused_modes
for m in "$@"; do
  AEC_FUSED_MODE=$m timeout -k 10 120 python $R/bench.py --no-cpu --no-c3 --no-rtf --steps 20 > $R/gpurun_out/fused_modes/m$m.log 2>&1 || exit 1
  echo "mode $m: $(tail -1 $R/gpurun_out/fused_modes/m$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel_ms_per_step"]; print(k.get("gru_synthesis", k.get("gru")))')"
done
AEC_FUSED_SYNTH=0 timeout -k 10 120 python $R/bench.py --no-cpu --no-c3 --no-rtf --steps 20 > $R/gpurun_out/fused_modes/unfused.log 2>&1 || exit 1
echo "unfused gru: $(tail -1 $R/gpurun_out/fused_modes/unfused.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel_ms_per_step"]; print(k.get("gru_synthesis", k.get("gru")))')"
