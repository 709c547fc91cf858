#!/usr/bin/env python3
"""profiles/pmc_latest_crn.json from a tools/crn_pmc_summary.py JSON (the
tools/crn_pmc.sh passes over tools/crn_probe.py --iters 1: two 256 x 10 s
batches).  bench.py reads `lstm_stage_hbm_bytes_per_batch` as the C3
roofline's `traffic`: the HBM bytes (2 x FETCH_SIZE + WRITE_SIZE, gfx950
correction) of the LSTM stage's kernels -- input projection GEMMs (the
M = 2 B T launches), persistent recurrences, combines -- per batch.

usage: crn_pmc_latest.py <summary.json> <source tag> [dtype]"""
import json
import sys

summ = json.load(open(sys.argv[1]))
tag = sys.argv[2]
dtype = sys.argv[3] if len(sys.argv) > 3 else 'bf16'
B, N = 256, 160000
T = N // 256 + 1
gemm_grid = str((2 * B * T + 255) // 256 * 32 * 512)     # 256x256 tiles, 8 waves, N = 8192
stage = {}
for k, v in summ.items():
    lstm = ('lstm_persist' in k or 'lstm_combine' in k or 'lstm_step' in k
            or (('gemm_rows_dma' in k or 'gemm_mx8' in k) and k.endswith('grid ' + gemm_grid)))
    if lstm:
        stage[k] = v
batches = 2
total = sum(v['hbm_bytes_per_launch'] * v['launches'] for v in stage.values())
out = dict(pipeline='crn', dtype=dtype, B=B, N=N,
           source=f'rocprofv3 --pmc passes (tools/crn_pmc.sh {tag}) over tools/crn_probe.py --iters 1 (2 batches)',
           formula='hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE = half of streamed bytes)',
           lstm_stage_kernels=stage,
           lstm_stage_hbm_bytes_per_batch=int(total / batches),
           kernels=summ)
json.dump(out, open('profiles/pmc_latest_crn.json', 'w'), indent=1)
print('lstm stage HBM bytes per batch', out['lstm_stage_hbm_bytes_per_batch'], 'from', len(stage), 'kernels')
