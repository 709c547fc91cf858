#!/bin/bash
# round-4 session-2 evidence: default bench line, C5 hop trace
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python $R/bench.py > $R/gpurun_out/r04p_bench.log 2>&1 || { echo "bench failed"; tail -20 $R/gpurun_out/r04p_bench.log; exit 1; }
echo "bench done"
bash $R/tools/c5_prof.sh r04p > $R/gpurun_out/r04p_c5prof.log 2>&1 || { echo "c5 prof failed"; tail -20 $R/gpurun_out/r04p_c5prof.log; exit 1; }
tail -3 $R/gpurun_out/r04p_c5prof.log
python $R/tools/c5_hop_table.py $R/gpurun_out/prof_r04p > $R/gpurun_out/r04p_c5_hop_table.txt && cat $R/gpurun_out/r04p_c5_hop_table.txt
