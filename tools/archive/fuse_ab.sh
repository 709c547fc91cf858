#!/bin/bash
# Fused look-ahead normaliser: the NLMS GPU tests, then the C2 line with AEC_PREP_FUSE 0 / 1 and
# look-ahead distance 1 / 2, alternating rounds (bench.py C2 only, 100 timed steps).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fuse_ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_nlms.py -x -q --timeout 300 --timeout-method thread \
    -m gpu > $O/nlms_tests.log 2>&1 || { echo "nlms tests failed"; tail -30 $O/nlms_tests.log; exit 1; }
tail -2 $O/nlms_tests.log
for r in 1 2 3; do
  for cfg in "0 1" "1 1" "1 2" "0 2"; do
    set -- $cfg
    AEC_PREP_FUSE=$1 timeout -k 10 200 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train \
        --lookahead $2 > $O/fuse$1_la$2_$r.log 2>&1 || { echo "bench failed"; tail -20 $O/fuse$1_la$2_$r.log; exit 1; }
    echo "round $r fuse=$1 lookahead=$2: $(tail -1 $O/fuse$1_la$2_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
  done
done
