#!/bin/bash
# Round 6: recurrence loop forms (A/B builds): h stored by both K halves (no exec-mask branch),
# full chunks unrolled; batch-1 / 64-stream latency and the C2 step, alternating on one box, then
# the fused-synthesis / pipeline bit-exactness tests on the last variant.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/rec_ab; mkdir -p $O
cd $R
export AEC_BENCH_AB=1
for i in 1 2 3; do
  for v in rec_base rec_st rec_full; do
    AEC_HIP_LIB=$R/ab_libs/$v.so timeout -k 10 120 python tools/b1_probe.py --sizes 1,64 --reps 20 > $O/${v}_b1_$i.log 2>&1 \
        || { tail -20 $O/${v}_b1_$i.log; exit 1; }
    AEC_HIP_LIB=$R/ab_libs/$v.so timeout -k 10 150 python bench.py --no-cpu --no-c3 --no-rtf --no-train --no-sweep \
        --steps 100 --warmup 5 > $O/${v}_c2_$i.log 2>&1 || { tail -20 $O/${v}_c2_$i.log; exit 1; }
    echo "$v #$i: b1 $(grep '"B": 1,' $O/${v}_b1_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_median"], d["out_sum"])') b64 $(grep '"B": 64,' $O/${v}_b1_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_median"], d["out_sum"])') c2 $(grep '^{' $O/${v}_c2_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("kernel_ms_per_step"))')"
  done
done
AEC_HIP_LIB=$R/ab_libs/rec_full.so timeout -k 10 300 python -u -m pytest tests/test_gpu_nlms.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "pipeline or split_path or fused_synthesis or batch_vs_oracle" > $O/rec_full_tests.log 2>&1 \
    || { tail -30 $O/rec_full_tests.log; exit 1; }
tail -1 $O/rec_full_tests.log
