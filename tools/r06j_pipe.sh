#!/bin/bash
# Round 6: the pipelined small-batch path (recursion + mic_erb in producer blocks of the GRU +
# synthesis launch): its bit-exactness tests, the NLMS / parity suites, then batch-1 / small-batch
# latency against the three-launch split path, and a kernel trace of B = 1.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_nlms.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "pipeline or split_path or fused_synthesis" > $O/r06j_pipe_test.log 2>&1 || { tail -40 $O/r06j_pipe_test.log; exit 1; }
grep -E 'PASS|FAIL' $O/r06j_pipe_test.log | tail -8
timeout -k 10 600 python -u -m pytest tests/test_gpu_nlms.py tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/r06j_gputest.log 2>&1 || { tail -30 $O/r06j_gputest.log; exit 1; }
tail -1 $O/r06j_gputest.log
for cfg in "" "AEC_SMALLB_PIPE=0"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/b1_probe.py --sizes 1,4,16,64 || exit 1
done
cd /tmp && export TMPDIR=/tmp
mkdir -p $O/b1 && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/b1/prof_pipe -o run -- python3 $R/tools/b1_probe.py --sizes 1 --reps 10 \
    > $O/b1/prof_pipe.log 2>&1 || { tail -20 $O/b1/prof_pipe.log; exit 1; }
echo profiled
