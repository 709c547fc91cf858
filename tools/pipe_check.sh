#!/bin/bash
# K6 pipeline: bit-exactness against the multi-kernel path, then bench both (round 2 A/B).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_nlms.py -k "pipeline or 10s" -x -v --timeout 200 --timeout-method thread > gpurun_out/pipe_tests.log 2>&1 || { tail -40 gpurun_out/pipe_tests.log; exit 1; }
tail -3 gpurun_out/pipe_tests.log
for pl in full postfilter; do
  for pipe in 1 0; do
    AEC_PIPE=$pipe timeout -k 10 200 python bench.py --pipeline $pl --steps 20 --warmup 3 --no-cpu --no-c3 > gpurun_out/b_${pl}_pipe${pipe}.json 2> gpurun_out/b_${pl}_pipe${pipe}.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/b_${pl}_pipe${pipe}.json'));print('$pl pipe=$pipe', d['ms_per_step'], d['kernel_ms_per_step'], d['rtf_batch1'])"
  done
done
