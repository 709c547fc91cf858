#!/usr/bin/env python3
"""Streaming DCCRN latency: B concurrent streams, one 256-sample hop per step
(hipGraph replay).  Prints per-hop latency and the real-time factor."""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
import aec_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--B', type=int, default=256)
ap.add_argument('--dtype', default='bf16')
ap.add_argument('--hops', type=int, default=200)
a = ap.parse_args()
torch.manual_seed(0)
net = aec_amd.dccrn2.DCCRN(aec_amd.net_conf, dtype=a.dtype).eval().cuda()
net.stream_open(a.B)
mic = 0.1 * torch.randn(a.B, 256, device='cuda')
far = 0.1 * torch.randn(a.B, 256, device='cuda')
out = torch.empty(a.B, 256, device='cuda')
with torch.no_grad():
    for _ in range(10):
        net.stream_step(mic, far, out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.hops):
        net.stream_step(mic, far, out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.hops
print(json.dumps(dict(B=a.B, dtype=a.dtype, ms_per_hop=round(dt * 1e3, 4), hop_ms=16.0,
                      rtf=round(dt / 0.016, 5), frames_per_s=round(a.B / dt, 1),
                      graph=os.environ.get('AEC_CRN_GRAPH', '1'))))
