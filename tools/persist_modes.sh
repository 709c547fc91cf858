#!/bin/bash
# Persistent LSTM recurrence: timing decomposition (CRN_PERSIST_MODE bits; results invalid unless 0).
set -o pipefail
mkdir -p gpurun_out
for m in ${MODES:-0 1 2 4 6 7}; do
  CRN_PERSIST_MODE=$m AEC_CRN_PERSIST=${PV:-1} timeout -k 10 300 python bench.py --pipeline crn --steps 3 --warmup 1 --no-cpu --no-rtf --inflight 1 > gpurun_out/pm_$m.json 2> gpurun_out/pm_$m.err || exit 1
  python - "$m" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/pm_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print('mode', sys.argv[1], d['ms_per_step'], d['stage_ms_per_step']['lstm'])
PY
done
