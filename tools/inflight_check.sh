#!/bin/bash
# Batches in flight (bench.py --inflight): 1 (sequential) vs 2 vs 3.
set -o pipefail
mkdir -p gpurun_out
for k in ${INFL:-1 2 3 2}; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-c3 --no-rtf --inflight $k > gpurun_out/infl_$k.json 2> gpurun_out/infl_$k.err || exit 1
  python - "$k" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/infl_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print('inflight', sys.argv[1], d['ms_per_step'], d['kernel_ms_per_step'], d['value'])
PY
done
