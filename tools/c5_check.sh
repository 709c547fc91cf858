#!/bin/bash
# CRN streaming checks + the C5 per-hop step timing (bench.py's run_c5_stream).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-c5}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_crn.py tests/test_gpu_crn_nlms.py -m gpu -q -k "stream" --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -c "
import sys, json; sys.argv=['bench.py']
import bench, torch
r = bench.run_c5_stream(torch.device('cuda', 0))
print(json.dumps(r))
" > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_c5.json').read().strip().splitlines()[-1]); print('C5 ms/hop', d['ms_per_hop'], 'frames/s', d['frames_per_s'])"
