#!/bin/bash
# Persistent LSTM recurrence: CRN parity tests (persistent path on), then the
# DCCRN bench with and without it (one batch in flight: the stage times are
# the kernels').
set -o pipefail
mkdir -p gpurun_out
AEC_CRN_PERSIST=${TESTV:-2} timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_crn.py tests/test_gpu_crn_nlms.py > gpurun_out/persist_tests.log 2>&1 || { tail -40 gpurun_out/persist_tests.log; exit 1; }
tail -3 gpurun_out/persist_tests.log
for k in ${PERSIST:-1 0}; do
  AEC_CRN_PERSIST=$k timeout -k 10 300 python bench.py --pipeline crn --steps 5 --warmup 2 --no-cpu --no-rtf --inflight 1 > gpurun_out/persist_b$k.json 2> gpurun_out/persist_b$k.err || exit 1
  python - "$k" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/persist_b{sys.argv[1]}.json').read().strip().splitlines()[-1])
print('AEC_CRN_PERSIST', sys.argv[1], d['ms_per_step'], d['stage_ms_per_step'])
PY
done
