#!/bin/bash
# round 5 batch t: with the new defaults (look-ahead, moments_lds, overlap-add on the recurrence
# waves): packed inverse FFT build and 3 batches in flight
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
AB=$R/acoustic-echo-cancellation_amd/aec_amd/ab
mkdir -p $O
for i in 1 2; do for v in "tree 2" "pkinv 2" "tree 3" "pkinv 3"; do
  set -- $v
  if [ $1 = tree ]; then unset AEC_HIP_LIB; else export AEC_HIP_LIB=$AB/$1.so; fi
  timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 40 --inflight $2 > $O/r05t_$1_$2_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05t_$1_$2_$i.log; exit 1; }
  echo "$1 inflight $2 #$i: $(tail -1 $O/r05t_$1_$2_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
done; done
bash $R/tools/r05_final_a.sh
