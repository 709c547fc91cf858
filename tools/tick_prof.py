#!/usr/bin/env python3
"""Per-tick role timing of nlms_analysis_kernel (a -DAEC_TICK_PROF build,
tools/build_variant.sh tick tree -DAEC_TICK_PROF, loaded via AEC_HIP_LIB):
runs the full pipeline at 256 x 10 s and prints, per role, the median over
ticks of work time and barrier waits (s_memtime cycles) for blocks 0 and 128.
  AEC_HIP_LIB=.../ab/tick.so python tools/tick_prof.py"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
import aec_amd  # noqa: E402
from aec_amd import _lib, synth  # noqa: E402

dev = torch.device('cuda', 0)
w = dict(np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz')))
net = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=aec_amd.nlms_conf).eval()
sd = net.state_dict()
for k in ['gru1.weight_ih_l0', 'gru1.weight_hh_l0', 'gru1.bias_ih_l0', 'gru1.bias_hh_l0',
          'linear1.weight', 'linear1.bias', 'linear2.weight', 'linear2.bias']:
    sd[k] = torch.from_numpy(w[k])
net.load_state_dict(sd)
net = net.to(dev)
erb = torch.tensor(aec_amd.erb_matrix(), dtype=torch.float32, device=dev)
B, n = 256, 160000
mic, ref, near = (torch.from_numpy(a).to(dev) for a in synth.batch(B, n, seed0=0))
with torch.no_grad():
    for _ in range(3):
        net.forward_ragged(mic, ref, near, erb, [n] * B)
torch.cuda.synchronize()
lib = _lib.load()
buf = np.zeros((2, 12, 48, 4), np.uint64)
rc = lib.aec_debug_tick_prof(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
assert rc == 0, rc
roles = ['mic', 'ref', 'nlms']
for blk in range(2):
    b = buf[blk].astype(np.int64)
    ticks = range(2, 40)
    tot = [b[0, c + 1, 0] - b[0, c, 0] for c in ticks]
    print(f'block {blk * 128}: tick period median {np.median(tot):.0f} cycles, total loop {b[0, 41, 3] - b[0, 0, 0]} cycles')
    for r in range(3):
        for q in range(4):
            wv = 4 * r + q
            work = np.median([b[wv, c, 1] - b[wv, c, 0] for c in ticks])
            w1 = np.median([b[wv, c, 2] - b[wv, c, 1] for c in ticks])
            mid = np.median([b[wv, c, 3] - b[wv, c, 2] for c in ticks])
            print(f'  {roles[r]:4s} wave {wv:2d}: work {work:7.0f}  wait b1 {w1:7.0f}  b1->b2 {mid:6.0f}')
