#!/bin/bash
# near=None (deployment form) on the GPU: the bit-exactness test, then the C2 step with and
# without near, the mic_erb pass on the ref waves (AEC_NLMS_ERB=1, round-6 kernel) against the mic
# waves (0, the default without near), alternating, A/B library of the working tree.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_nlms.py -x -v --timeout 120 --timeout-method thread \
    -k "no_near or lookahead or batch_invariance" > $O/r06t_test.log 2>&1 || { tail -30 $O/r06t_test.log; exit 1; }
tail -2 $O/r06t_test.log
for i in 1 2 3; do
  for e in 0 1; do
    AEC_HIP_LIB=$R/ab_libs/ab_tree.so AEC_BENCH_AB=1 AEC_NLMS_ERB=$e timeout -k 10 240 \
        python bench.py --steps 100 --warmup 5 --no-c3 --no-train --no-cpu --no-sweep --no-rtf > $O/r06t_b.log 2>&1 \
        || { tail -20 $O/r06t_b.log; exit 1; }
    python - "$e" $O/r06t_b.log <<'PY' | tee -a $O/r06t_nonear_ab.log
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
print(f"AEC_NLMS_ERB={sys.argv[1]}  with near {d['ms_per_step']} ms  no near {d['no_near']['ms_per_step']} ms "
      f"({d['no_near']['frames_per_s'] / 1e6:.1f} M frames/s)")
PY
  done
done
