#!/usr/bin/env python3
"""Streaming Little_net latency (include/aec_hip.h aec_stream_step): B
concurrent streams, one 256-sample hop per call = one fused kernel launch
(STFT -> [FD-NLMS] -> ERB -> GRU step -> head -> iSTFT / OLA).  Prints the
per-hop wall time (host loop, device-synchronised at the end), the HIP-event
kernel time per hop and the real-time factor."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
import aec_amd  # noqa: E402
from aec_amd.erb import EquivalentRectangularBandwidth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--B', type=int, default=256)
ap.add_argument('--taps', type=int, default=4, help='NLMS taps (0 = post-filter only)')
ap.add_argument('--hops', type=int, default=500)
a = ap.parse_args()
torch.manual_seed(0)
nlms = dict(aec_amd.nlms_conf, taps=a.taps) if a.taps else None
net = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=nlms).eval().cuda()
erb = torch.tensor(EquivalentRectangularBandwidth(257, 16000, 32, 0, 8000).filters, dtype=torch.float32).cuda()
net.stream_open(a.B, erb)
mic = 0.1 * torch.randn(a.B, 256, device='cuda')
far = 0.1 * torch.randn(a.B, 256, device='cuda')
with torch.no_grad():
    for _ in range(20):
        net.stream_step(mic, far)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.hops):
        net.stream_step(mic, far)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.hops
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ks = []
    for _ in range(50):
        e0.record()
        net.stream_step(mic, far)
        e1.record()
        e1.synchronize()
        ks.append(e0.elapsed_time(e1))
print(json.dumps(dict(B=a.B, nlms_taps=a.taps, ms_per_hop=round(dt * 1e3, 4),
                      event_ms_per_hop_median=round(float(np.median(ks)), 4), hop_ms=16.0,
                      rtf=round(dt / 0.016, 5), frames_per_s=round(a.B / dt, 1))))
