#!/bin/bash
# Round 6: NS chosen by batch size (NS = 1 up to half the CUs): small-batch latency against the
# forced NS = 2, the NLMS / parity GPU tests, the bench line.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
cd $R
for cfg in "" "AEC_GRU_NS=2"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/b1_probe.py --sizes 1,16,64,128,129,256 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_nlms.py tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/r06i_gputest.log 2>&1 || { tail -30 $O/r06i_gputest.log; exit 1; }
tail -2 $O/r06i_gputest.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-c3 --no-train > $O/r06i_bench.log 2>&1 || { tail -30 $O/r06i_bench.log; exit 1; }
grep '^{' $O/r06i_bench.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["rtf_batch1"], d.get("batch_sweep_frames_per_s"))'
