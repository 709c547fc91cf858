#!/bin/bash
# round-5 end-of-round evidence (4/4, after the C5 direct-launch default): GPU suite, smoke,
# default bench line, C5 per-hop trace and hop table
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/r05zz_gputest.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error" $O/r05zz_gputest.log | head; tail -30 $O/r05zz_gputest.log; exit 1; }
tail -1 $O/r05zz_gputest.log
cp $O/parity_margins.json $O/r05zz_parity_margins.json
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05zz_smoke.log 2>&1 || { echo "smoke failed"; tail $O/r05zz_smoke.log; exit 1; }
tail -1 $O/r05zz_smoke.log
timeout -k 10 500 python $R/bench.py > $O/r05zz_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/r05zz_bench.log; exit 1; }
tail -1 $O/r05zz_bench.log | head -c 300; echo
bash $R/tools/c5_prof.sh r05zz_c5 > $O/r05zz_c5prof.log 2>&1 || { echo "c5 trace failed"; tail $O/r05zz_c5prof.log; exit 1; }
python $R/tools/c5_hop_table.py $O/prof_r05zz_c5 > $O/r05zz_c5_hop_table.txt 2>&1 || exit 1
cat $O/r05zz_c5_hop_table.txt
