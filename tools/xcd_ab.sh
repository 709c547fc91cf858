#!/bin/bash
# Row / MX GEMM tile order (CRN_GEMM_XCD) A/B on one box, alternating:
#   bash tools/xcd_ab.sh "0 4 8" [rounds] -> C3 probe stage line and C5 ms per hop per value
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
VALS=${1:-"0 4 8"}; ROUNDS=${2:-2}
mkdir -p $R/gpurun_out/xcd_ab
for r in $(seq 1 $ROUNDS); do
  for v in $VALS; do
    CRN_GEMM_XCD=$v timeout -k 10 180 python $R/tools/crn_probe.py --skip-golden --iters 3 > $R/gpurun_out/xcd_ab/c3_${v}_$r.log 2>&1 || exit 1
    echo "round $r CRN_GEMM_XCD=$v C3: $(tail -1 $R/gpurun_out/xcd_ab/c3_${v}_$r.log)"
  done
done
bash $R/tools/c5_ab_env.sh $ROUNDS $(for v in $VALS; do echo CRN_GEMM_XCD=$v; done) || exit 1
