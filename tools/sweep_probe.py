#!/usr/bin/env python3
"""Per-kernel HIP-event times of the full pipeline (NLMS -> GRU post-filter)
at several stream counts (the bench line's batch sweep, one batch in flight):
python tools/sweep_probe.py [B ...]"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
import aec_amd  # noqa: E402
from aec_amd import synth  # noqa: E402

dev = torch.device('cuda', 0)
w = dict(np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz')))
net = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=aec_amd.nlms_conf).eval()
sd = net.state_dict()
for k in w:
    if k in sd and not k.startswith(('cpx_stft', 'istft')):
        sd[k] = torch.from_numpy(w[k])
net.load_state_dict(sd)
net = net.to(dev)
erb = torch.tensor(aec_amd.erb_matrix(), dtype=torch.float32, device=dev)
n = 160000
T = n // 256 + 1
mic, ref, near = (torch.from_numpy(a).to(dev) for a in synth.batch(256, n, seed0=0))
Bs = [int(x) for x in sys.argv[1:]] or [256, 512, 768, 1024, 1280, 2048, 4096]
for bb in Bs:
    rep = (bb + 255) // 256
    mm, rr, nn_ = (x.repeat(rep, 1)[:bb].contiguous() for x in (mic, ref, near))
    with torch.no_grad():
        net.forward_ragged(mm, rr, nn_, erb, [n] * bb)
        torch.cuda.synchronize()
        h = net._handle(dev)[0]
        h.profile_enable(True)
        for _ in range(3):
            net.forward_ragged(mm, rr, nn_, erb, [n] * bb)
        torch.cuda.synchronize()
        kms, calls = h.profile_read()
        h.profile_enable(False)
        t1 = time.perf_counter()
        for _ in range(3):
            net.forward_ragged(mm, rr, nn_, erb, [n] * bb)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t1) / 3
    per = [k / max(calls, 1) for k in kms]
    print(f'B={bb:5d} ms/call {el*1e3:8.3f} frames/s {bb*T/el/1e6:8.2f} M  kernels ms '
          + ' '.join(f'{x:.3f}' for x in per) + f'  per 256 streams {el*1e3*256/bb:.3f}', flush=True)
    del mm, rr, nn_
    torch.cuda.empty_cache()
