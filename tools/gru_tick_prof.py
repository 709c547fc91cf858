#!/usr/bin/env python3
"""Per-tick role timing of gru_synth_kernel (a -DAEC_TICK_PROF build loaded via
AEC_HIP_LIB): the full pipeline at B x 10 s (default 256), then per wave the
median over ticks of the work time (loop top -> before the tick barrier) and of
the tick period, (consumer) blocks 0 and 64 (s_memtime cycles), and when each
wave reached its first ticks relative to the recurrence wave's first stamp.
  AEC_HIP_LIB=.../ab_libs/tick.so python tools/gru_tick_prof.py [--streams B]"""
import argparse
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
ap = argparse.ArgumentParser()
ap.add_argument('--streams', type=int, default=256)
a = ap.parse_args()
B, n = a.streams, 160000
mic, ref, near = (torch.from_numpy(a).to(dev) for a in synth.batch(B, n, seed0=0))
with torch.no_grad():
    for _ in range(3):
        net.forward_ragged(mic, ref, near, erb, [n] * B)
torch.cuda.synchronize()
lib = _lib.load()
buf = np.zeros((2, 12, 96, 2), np.uint64)
rc = lib.aec_debug_gru_tick_prof(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
assert rc == 0, rc
ns = int(os.environ.get('AEC_GRU_NS', '0')) or (1 if 2 * B <= 256 else 2)     # launch_gru_synth's rule
roles = ['rec'] * ns + ['gi'] * 3 + ['head'] * 3 + ['synth'] * 4
nticks = (n // 256 + 1 + 16 // ns - 1) // (16 // ns) + 6
for blk in range(2 if B > 64 * ns else 1):
    b = buf[blk].astype(np.int64)
    ticks = range(6, min(80, nticks - 4))
    t0 = b[0, 0, 0]
    print('  first stamps (cycles after rec wave tick -3):',
          {roles[w] + str(w): [int(b[w, c, 0] - t0) for c in range(0, 6)] for w in range(len(roles))})
    per = [b[0, c + 1, 0] - b[0, c, 0] for c in ticks]
    print(f'block {blk * 64}: tick period median {np.median(per):.0f} cycles')
    for wv in range(len(roles)):
        work = np.median([b[wv, c, 1] - b[wv, c, 0] for c in ticks])
        print(f'  {roles[wv]:5s} wave {wv:2d}: work {work:7.0f}')
