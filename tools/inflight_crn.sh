#!/bin/bash
# DCCRN (C3) with 1 vs 2 batches in flight, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 300 python bench.py --pipeline crn --steps 10 --warmup 2 --no-cpu --no-rtf --crn-inflight $k > gpurun_out/inflc_$k.json 2> gpurun_out/inflc_$k.err || exit 1
  python - "$k" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/inflc_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print('crn inflight', sys.argv[1], d['ms_per_step'], d['stage_ms_per_step'], d['value'])
PY
done
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
tail -c 3000 gpurun_out/bench_default.json
