#!/bin/bash
# round 5 batch v: C2 batches in flight 2 / 3 / 4 at 100 timed steps (look-ahead on)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for i in 1 2 3; do for f in 2 3 4; do
  timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 100 --inflight $f > $O/r05v_if${f}_$i.log 2>&1 || { echo "bench $f failed"; tail -5 $O/r05v_if${f}_$i.log; exit 1; }
  echo "inflight $f #$i: $(tail -1 $O/r05v_if${f}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done; done
# the synthesis window applied in the recurrence waves' overlap-add (-DAEC_OLA_WIN=1): bit identity,
# C2 A/B at 100 steps, gru tick profile
AB=$R/acoustic-echo-cancellation_amd/aec_amd/ab
for lib in tree olawin; do
  if [ $lib = tree ]; then unset AEC_HIP_LIB; else export AEC_HIP_LIB=$AB/$lib.so; fi
  echo "$lib: $(timeout -k 10 120 python $R/tools/lib_bitcmp.py 2>&1 | grep sha1)"
done
for i in 1 2 3; do for lib in tree olawin; do
  if [ $lib = tree ]; then unset AEC_HIP_LIB; else export AEC_HIP_LIB=$AB/$lib.so; fi
  timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 100 > $O/r05v_${lib}_$i.log 2>&1 || { echo "bench $lib failed"; exit 1; }
  echo "$lib #$i: $(tail -1 $O/r05v_${lib}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
done; done
AEC_HIP_LIB=$AB/tick_olawin.so timeout -k 10 120 python $R/tools/gru_tick_prof.py > $O/r05v_gru_tick_olawin.txt 2>&1 || { echo "gru tick failed"; exit 1; }
head -14 $O/r05v_gru_tick_olawin.txt
