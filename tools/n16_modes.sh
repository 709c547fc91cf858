#!/bin/bash
# 16-wave NLMS analysis: timing decomposition (AEC_NLMS_MODE bits) and wave priorities.
set -o pipefail
mkdir -p gpurun_out
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-c3 --no-rtf > gpurun_out/n16m_$lab.json 2> gpurun_out/n16m_$lab.err || exit 1
  python - "$lab" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/n16m_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], d['kernel_ms_per_step'].get('analysis'))
PY
}
for m in ${MODES:-0 1 2 4 8 6 14}; do run "k16_mode$m" AEC_NLMS16=1 AEC_NLMS_MODE=$m; done
for pr in ${PRIOS:-1 2 1111 2221}; do run "k16_prio$pr" AEC_NLMS16=1 AEC_NLMS_PRIO=$pr; done
run k12 AEC_NLMS16=0
