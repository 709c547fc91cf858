#!/bin/bash
# round-5 end-of-round evidence (2/3): C2 rocprofv3 trace + FETCH / WRITE passes (one batch in
# flight), SQ counter passes, NLMS-analysis and gru_synth tick profiles of the final build
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
AB=$R/acoustic-echo-cancellation_amd/aec_amd/ab
mkdir -p $O
for i in 1 2; do for k in 20 100; do
  timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps $k > $O/r05z_steps_${k}_$i.log 2>&1 || { echo "bench steps $k failed"; exit 1; }
  echo "steps $k #$i: $(tail -1 $O/r05z_steps_${k}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done; done
bash $R/tools/profile.sh r05z_full --inflight 1 > $O/r05z_profile.log 2>&1 || { echo "profile failed"; tail $O/r05z_profile.log; exit 1; }
echo "profile done"
bash $R/tools/sq_pmc.sh r05z_sq > $O/r05z_sq.log 2>&1 || { echo "sq failed"; tail $O/r05z_sq.log; exit 1; }
echo "sq done"
AEC_HIP_LIB=$AB/tick.so timeout -k 10 120 python $R/tools/tick_prof.py > $O/r05z_nlms_tick.txt 2>&1 || { echo "nlms tick failed"; tail $O/r05z_nlms_tick.txt; exit 1; }
head -14 $O/r05z_nlms_tick.txt
AEC_HIP_LIB=$AB/tick.so timeout -k 10 120 python $R/tools/gru_tick_prof.py > $O/r05z_gru_tick.txt 2>&1 || { echo "gru tick failed"; tail $O/r05z_gru_tick.txt; exit 1; }
head -14 $O/r05z_gru_tick.txt
