#!/bin/bash
# K6 timing decomposition: AEC_PIPE_MODE bit r skips role r's work (results invalid unless 0).
set -o pipefail
mkdir -p gpurun_out
for mode in ${MODES:-0 1 2 4 8 16 32 64 128 176 240 255 254}; do
  AEC_PIPE_MODE=$mode timeout -k 10 120 python bench.py --pipeline full --steps 20 --warmup 3 --no-cpu --no-c3 > gpurun_out/pm_$mode.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/pm_$mode.json'));print('mode $mode', d['ms_per_step'], d['kernel_ms_per_step'].get('analysis'), 'rtf1', d['rtf_batch1'])"
done
