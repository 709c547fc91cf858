#!/bin/bash
# round-5 end-of-round evidence (5/5, window in the overlap-add by default): GPU suite, smoke,
# default bench line, gru_synth and NLMS tick profiles
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
AB=$R/acoustic-echo-cancellation_amd/aec_amd/ab
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/r05zf_gputest.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error" $O/r05zf_gputest.log | head; tail -30 $O/r05zf_gputest.log; exit 1; }
tail -1 $O/r05zf_gputest.log
cp $O/parity_margins.json $O/r05zf_parity_margins.json
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05zf_smoke.log 2>&1 || { echo "smoke failed"; tail $O/r05zf_smoke.log; exit 1; }
tail -1 $O/r05zf_smoke.log
timeout -k 10 500 python $R/bench.py > $O/r05zf_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/r05zf_bench.log; exit 1; }
tail -1 $O/r05zf_bench.log | head -c 300; echo
AEC_HIP_LIB=$AB/tick.so timeout -k 10 120 python $R/tools/gru_tick_prof.py > $O/r05zf_gru_tick.txt 2>&1 || { echo "gru tick failed"; exit 1; }
head -14 $O/r05zf_gru_tick.txt
bash $R/tools/profile.sh r05zf_full --inflight 1 > $O/r05zf_profile.log 2>&1 || { echo "profile failed"; tail $O/r05zf_profile.log; exit 1; }
echo "profile done"
