#!/bin/bash
# Fused look-ahead normaliser, second form (buffer descriptors): NLMS GPU tests, then the C2 line
# for the previous HEAD library (ab/head.so), this build unfused (AEC_PREP_FUSE=0) and fused at
# look-ahead distance 2, alternating rounds; then a kernel trace of the fused configuration.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fuse_ab2
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_nlms.py -x -q --timeout 300 --timeout-method thread \
    -m gpu > $O/nlms_tests.log 2>&1 || { echo "nlms tests failed"; tail -30 $O/nlms_tests.log; exit 1; }
tail -1 $O/nlms_tests.log
B="--no-cpu --no-c3 --no-rtf --no-sweep --no-train"
for r in 1 2 3; do
  for cfg in head:0:1 new:0:1 new:1:2 new:1:3; do
    IFS=: read lib fu la <<< "$cfg"
    if [ $lib = head ]; then L=$R/acoustic-echo-cancellation_amd/aec_amd/ab/head.so; else L=; fi
    AEC_HIP_LIB=$L AEC_PREP_FUSE=$fu timeout -k 10 200 python $R/bench.py $B --lookahead $la --inflight 3 \
        > $O/${lib}_f${fu}_la${la}_$r.log 2>&1 || { echo "bench failed"; tail -20 $O/${lib}_f${fu}_la${la}_$r.log; exit 1; }
    echo "round $r $lib fuse=$fu la=$la: $(tail -1 $O/${lib}_f${fu}_la${la}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
  done
done
cd /tmp && export TMPDIR=/tmp
AEC_PREP_FUSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o fused -- python3 $R/bench.py $B \
    --lookahead 2 --steps 20 > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cat {} \; | head -12
