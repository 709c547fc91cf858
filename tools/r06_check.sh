#!/bin/bash
# Round-6 check on the GPU box: the GPU suite, smoke, and the default bench line.
#   tools/r06_check.sh <tag> [pytest -k expr]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06a}
K=${2:-}
O=$R/gpurun_out
mkdir -p $O
cd $R
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" \
      > $O/${TAG}_gputest.log 2>&1 || { tail -30 $O/${TAG}_gputest.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > $O/${TAG}_gputest.log 2>&1 || { tail -30 $O/${TAG}_gputest.log; exit 1; }
fi
tail -3 $O/${TAG}_gputest.log
cp -f $O/parity_margins.json $O/${TAG}_parity_margins.json 2>/dev/null
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { cat $O/${TAG}_smoke.log; exit 1; }
tail -1 $O/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/${TAG}_bench.log 2>&1 || { tail -30 $O/${TAG}_bench.log; exit 1; }
grep '^{' $O/${TAG}_bench.log > $O/${TAG}_bench.json
python - "$O/${TAG}_bench.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
c5 = d['c5_stream_fp8']
print('C2 ms', d['ms_per_step'], 'value', d['value'], 'frac', d['roofline']['frac'], 'fp32_frac', d['pipeline_roofline']['fp32_frac'])
print('C3', d['c3_crn_bf16']['ms_per_step'], 'C3fp8', d['c3_crn_fp8']['ms_per_step'], 'C4', d['c4_nlms_crn_bf16_per_gpu']['ms_per_step'],
      'C4 cpu', (d['c4_nlms_crn_bf16_per_gpu'].get('cpu_baseline') or {}).get('value'))
print('C5 direct', c5['ms_per_hop'], 'graph', c5['graph_ms_per_hop'], c5['graph_stats'])
print('knobs', d['knobs'])
EOF
