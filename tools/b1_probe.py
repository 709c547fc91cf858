#!/usr/bin/env python3
"""Batch-1 / small-batch latency of the C2 path (bench.py's net: NLMS front, golden GRU weights):
median synchronous forward_ragged time over --reps calls per batch size, one JSON line per size.
Mode knobs (AEC_FUSED_SYNTH, AEC_GRU_NS, AEC_SMALLB) are read when the handle is created, so one
process measures one setting.
  python tools/b1_probe.py [--sizes 1,16,64] [--reps 20] [--seconds 10]"""
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
from aec_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--sizes', default='1,16,64')
ap.add_argument('--reps', type=int, default=20)
ap.add_argument('--seconds', type=float, default=10.0)
ap.add_argument('--bypass', action='store_true', help='no FD-NLMS (the reference-parity drop-in path)')
a = ap.parse_args()
dev = torch.device('cuda', 0)
w = dict(np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz')))
net = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=None if a.bypass else aec_amd.nlms_conf).eval()
sd = net.state_dict()
for k in ['gru1.weight_ih_l0', 'gru1.weight_hh_l0', 'gru1.bias_ih_l0', 'gru1.bias_hh_l0',
          'linear1.weight', 'linear1.bias', 'linear2.weight', 'linear2.bias']:
    sd[k] = torch.from_numpy(w[k])
net.load_state_dict(sd)
net = net.to(dev)
erb = torch.tensor(aec_amd.erb_matrix(), dtype=torch.float32, device=dev)
n = int(round(a.seconds * 16000))
env = {k: v for k, v in os.environ.items() if k.startswith(('AEC_', 'CRN_'))}
for B in [int(x) for x in a.sizes.split(',')]:
    mic, ref, near = (torch.from_numpy(x).to(dev) for x in synth.batch(B, n, seed0=0))
    lat = []
    with torch.no_grad():
        for i in range(a.reps + 3):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            out, loss = net.forward_ragged(mic, ref, near, erb, [n] * B)
            torch.cuda.synchronize(dev)
            if i >= 3:
                lat.append(time.perf_counter() - t0)
    ms = float(np.median(lat)) * 1e3
    print(json.dumps(dict(B=B, bypass=a.bypass, env=env, ms_median=round(ms, 4), ms_min=round(min(lat) * 1e3, 4),
                          frames_per_s=round(B * (n // 256 + 1) / ms * 1e3, 1), rtf=round(ms / 1e3 / a.seconds, 8),
                          out_sum=float(out.double().sum()), loss=float(loss.double().sum()))), flush=True)
