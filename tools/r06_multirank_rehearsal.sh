#!/bin/bash
# The N>1 bench flow on a one-GPU box: 2 ranks launched as the driver launches them
# (torch.distributed.run, 127.0.0.1), both on cuda:0, gloo for the barriers / max-over-ranks
# (AEC_BENCH_BACKEND=gloo; never used for numbers).  Checks that rank 0 prints one JSON line
# with n_gpus 2 and the C5 leg ran on every rank.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
AEC_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 \
    > gpurun_out/r06_multirank.log 2>&1 || { tail -30 gpurun_out/r06_multirank.log; exit 1; }
grep '^{' gpurun_out/r06_multirank.log > gpurun_out/r06_multirank.json
python - <<'PY'
import json
lines = open('gpurun_out/r06_multirank.json').read().splitlines()
assert len(lines) == 1, len(lines)
d = json.loads(lines[0])
assert d['n_gpus'] == 2, d['n_gpus']
print('n_gpus', d['n_gpus'], 'value', d['value'], 'per gpu', d['value_per_gpu'], 'ms', d['ms_per_step'],
      'c5 streams', d['c5_stream_fp8']['streams'], 'c5 ms/hop', d['c5_stream_fp8']['ms_per_hop'])
PY
