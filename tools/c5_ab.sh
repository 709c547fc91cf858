#!/bin/bash
# A/B of the C5 per-hop step over env settings: bash tools/c5_ab.sh "VAR=a" "VAR=b VAR2=c" ...
# (the first run is the default build; TESTS=1 runs the streaming parity tests once first)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-c5ab}
mkdir -p $R/gpurun_out
cd $R
if [ "${TESTS:-0}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_crn.py tests/test_gpu_crn_nlms.py -m gpu -q -k "stream" --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.log
fi
i=0
for cfg in "base" "$@"; do
  i=$((i+1))
  envs=""; [ "$cfg" != "base" ] && envs="$cfg"
  env $envs timeout -k 10 200 python -c "
import sys, json; sys.argv=['bench.py']
import bench, torch
r = bench.run_c5_stream(torch.device('cuda', 0))
print(json.dumps(r))
" > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_$i.json').read().strip().splitlines()[-1]); print('$cfg', 'C5 ms/hop', d['ms_per_hop'])"
done
