#!/bin/bash
# round 5: window in the recurrence waves' overlap-add, products through inline asm (no contraction
# into the add): bit identity against HEAD, the fused-synthesis tests on that build, C2 A/B
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
AB=$R/acoustic-echo-cancellation_amd/aec_amd/ab
mkdir -p $O
for lib in tree olawin; do
  if [ $lib = tree ]; then unset AEC_HIP_LIB; else export AEC_HIP_LIB=$AB/$lib.so; fi
  echo "$lib: $(timeout -k 10 120 python $R/tools/lib_bitcmp.py 2>&1 | grep sha1)"
done
AEC_HIP_LIB=$AB/olawin.so timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_nlms.py -m gpu -x -q -k "fused_synthesis or small_batch or lookahead" --timeout 240 --timeout-method thread > $O/r05z2_tests.log 2>&1; tail -3 $O/r05z2_tests.log
for i in 1 2 3; do for lib in tree olawin; do
  if [ $lib = tree ]; then unset AEC_HIP_LIB; else export AEC_HIP_LIB=$AB/$lib.so; fi
  timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train > $O/r05z2_${lib}_$i.log 2>&1 || { echo "bench $lib failed"; exit 1; }
  echo "$lib #$i: $(tail -1 $O/r05z2_${lib}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
done; done
