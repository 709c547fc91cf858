#!/usr/bin/env python3
"""Host-side cost of one forward_ragged call: synchronous wall time of a 1-hop call (B = 1, n = 256:
the kernels have almost nothing to do) against the GPU time of its kernels (HIP events around the
call), and a Python profile of the call.
  python tools/host_overhead_probe.py"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
import aec_amd  # noqa: E402
from aec_amd import synth  # noqa: E402

dev = torch.device('cuda', 0)
net = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=aec_amd.nlms_conf).eval().to(dev)
erb = torch.tensor(aec_amd.erb_matrix(), dtype=torch.float32, device=dev)
for n in (256, 160000):
    mic, ref, near = (torch.from_numpy(x).to(dev) for x in synth.batch(1, n, seed0=0))
    lat, gpu, call = [], [], []
    with torch.no_grad():
        for i in range(60):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            e0.record()
            net.forward_ragged(mic, ref, near, erb, [n])
            t1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            if i >= 10:
                lat.append(t2 - t0)
                call.append(t1 - t0)
                gpu.append(e0.elapsed_time(e1) * 1e-3)
    print(f'n={n}: wall {np.median(lat) * 1e6:.1f} us, host call returns after {np.median(call) * 1e6:.1f} us, '
          f'GPU (events) {np.median(gpu) * 1e6:.1f} us', flush=True)
mic, ref, near = (torch.from_numpy(x).to(dev) for x in synth.batch(1, 256, seed0=0))
pr = cProfile.Profile()
with torch.no_grad():
    pr.enable()
    for _ in range(200):
        net.forward_ragged(mic, ref, near, erb, [256])
    pr.disable()
torch.cuda.synchronize(dev)
pstats.Stats(pr).sort_stats('tottime').print_stats(18)
