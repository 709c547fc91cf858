#!/usr/bin/env python3
"""SHA-1 of the NLMS pipeline's outputs (waveform, loss, mic / ref / est features) on ragged
lengths with the library AEC_HIP_LIB points at (default: the in-tree build), so two builds
that must be bit-identical can be compared from two processes:
  AEC_HIP_LIB=.../ab/x.so python tools/lib_bitcmp.py   -> one line 'sha1 <hex> <what>'"""
import hashlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
import aec_amd  # noqa: E402
from aec_amd import synth  # noqa: E402

w = dict(np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz')))
net = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=aec_amd.nlms_conf).eval()
sd = net.state_dict()
for k in ['gru1.weight_ih_l0', 'gru1.weight_hh_l0', 'gru1.bias_ih_l0', 'gru1.bias_hh_l0',
          'linear1.weight', 'linear1.bias', 'linear2.weight', 'linear2.bias']:
    sd[k] = torch.from_numpy(w[k])
net.load_state_dict(sd)
net = net.to('cuda:0')
net.set_debug(True)
erb = torch.tensor(aec_amd.erb_matrix(), dtype=torch.float32, device='cuda:0')
lens = [160000, 33333, 4097, 255, 16000, 256, 159999, 70001] * 10      # 80 streams: the batch K2n path
L = max(lens)
rows = [synth.scene(n, 300 + i) for i, n in enumerate(lens)]
M, R, N = (np.zeros((len(lens), L), np.float32) for _ in range(3))
for i, (m, r, nn_) in enumerate(rows):
    M[i, :lens[i]], R[i, :lens[i]], N[i, :lens[i]] = m, r, nn_
M, R, N = (torch.tensor(a, device='cuda:0') for a in (M, R, N))
with torch.no_grad():
    out, loss = net.forward_ragged(M, R, N, erb, lens)
T = L // 256 + 1
h = hashlib.sha1()
h.update(out.cpu().numpy().tobytes())
h.update(loss.cpu().numpy().tobytes())
for k in ('mic_erb', 'ref_erb', 'est_erb'):
    f = net.debug_intermediate(k, len(lens), T).cpu().numpy()
    for i, n in enumerate(lens):
        h.update(f[i, :n // 256 + 1].tobytes())
if os.environ.get('LIB_BITCMP_DUMP'):   # the arrays themselves, to locate a difference
    np.savez(os.environ['LIB_BITCMP_DUMP'], out=out.cpu().numpy(), loss=loss.cpu().numpy())
print('sha1', h.hexdigest(), 'out/loss/mic_erb/ref_erb/est_erb of', len(lens), 'ragged streams,',
      os.path.basename(os.environ.get('AEC_HIP_LIB', 'libaec_hip.so')))
