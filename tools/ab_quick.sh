#!/bin/bash
# Quick A/B of the headline step: NLMS/parity GPU tests, then the C2 bench line (no CPU / C3 / training legs)
# once per env setting given as arguments (e.g. "AEC_NLMS_ERB=1").
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-ab}
mkdir -p $R/gpurun_out
cd $R
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_nlms.py tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_api.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.log
fi
i=0
for cfg in "base" "$@"; do
  i=$((i+1))
  envs=""; [ "$cfg" != "base" ] && envs="$cfg"
  env $envs timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu --no-c3 --no-train --no-sweep > gpurun_out/${TAG}_b$i.json 2> gpurun_out/${TAG}_b$i.err || { tail -20 gpurun_out/${TAG}_b$i.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/${TAG}_b$i.json') if l.startswith('{')][-1]); print('$cfg', d['ms_per_step'], d['kernel_ms_per_step'], d['rtf_batch1'])"
done
