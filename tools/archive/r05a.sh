#!/bin/bash
# round-5 first GPU batch: GPU suite (parity margins recorded), smoke, default bench line,
# C2 "before" evidence: per-tick role timing (AEC_TICK_PROF build) and two SQ counter passes
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 240 --timeout-method thread -s > $O/r05a_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/r05a_gputest.log; exit 1; }
tail -1 $O/r05a_gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05a_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/r05a_smoke.log
timeout -k 10 600 python $R/bench.py > $O/r05a_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/r05a_bench.log; exit 1; }
echo "bench done"
AEC_HIP_LIB=$R/acoustic-echo-cancellation_amd/aec_amd/ab/tick.so timeout -k 10 120 python $R/tools/tick_prof.py > $O/r05a_tick_profile.txt 2>&1 || { echo "tick prof failed"; exit 1; }
echo "tick done"
bash $R/tools/sq_pmc.sh r05a_before > $O/r05a_sq.log 2>&1 || { echo "sq failed"; exit 1; }
echo "sq done"
