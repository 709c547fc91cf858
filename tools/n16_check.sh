#!/bin/bash
# 16-wave NLMS analysis: bit-exactness vs the 12-wave kernel, then A/B timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nlms.py -k "nlms16 or 10s" > gpurun_out/n16_tests.log 2>&1 || { tail -30 gpurun_out/n16_tests.log; exit 1; }
tail -3 gpurun_out/n16_tests.log
for k in 0 1 0 1; do
  AEC_NLMS16=$k timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-c3 --no-rtf > gpurun_out/n16_b$k.json 2> gpurun_out/n16_b$k.err || exit 1
  python - "$k" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/n16_b{sys.argv[1]}.json').read().strip().splitlines()[-1])
print('AEC_NLMS16', sys.argv[1], d['ms_per_step'], d['kernel_ms_per_step'])
PY
done
