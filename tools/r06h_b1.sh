#!/bin/bash
# Round 6: batch-1 / small-batch latency of the C2 path per GRU + synthesis mode, then kernel
# traces of B = 1 for the default and the unfused path.
#   bash tools/r06h_b1.sh
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/b1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in "" "AEC_FUSED_SYNTH=0" "AEC_GRU_NS=1" "AEC_SMALLB=0" "AEC_FUSED_SYNTH=0 AEC_SMALLB=0"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python $R/tools/b1_probe.py --sizes 1,4,16,64,128 || exit 1
done
for cfg in default unfused; do
  if [ $cfg = unfused ]; then export AEC_FUSED_SYNTH=0; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_$cfg -o run -- python3 $R/tools/b1_probe.py --sizes 1 --reps 10 \
      > $O/prof_$cfg.log 2>&1 || { tail -20 $O/prof_$cfg.log; exit 1; }
done
find $O -name '*kernel_stats.csv' | while read f; do echo "== $f"; cut -d, -f1-4 "$f" | head -12; done
