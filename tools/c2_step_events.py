#!/usr/bin/env python3
"""Where the C2 timed region's fixed overhead goes: the bench's own loop (bench.py, three or two
batches in flight, normaliser look-ahead) with a HIP event recorded on each step's stream after
its kernels, so each batch's completion time relative to the region's start is visible.

  python tools/c2_step_events.py [--steps 20] [--warmup 5] [--inflight 2] [--lookahead 1]"""
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
ap.add_argument('--steps', type=int, default=20)
ap.add_argument('--warmup', type=int, default=5)
ap.add_argument('--inflight', type=int, default=2)
ap.add_argument('--lookahead', type=int, default=1)
ap.add_argument('--paced', type=int, default=1, help='bench.py\'s pacing of the look-ahead passes')
a = ap.parse_args()
dev = torch.device('cuda', 0)
B, n = 256, 160000
w = dict(np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz')))
nets = []
for _ in range(a.inflight):
    net = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=aec_amd.nlms_conf).eval()
    sd = net.state_dict()
    for k in ['gru1.weight_ih_l0', 'gru1.weight_hh_l0', 'gru1.bias_ih_l0', 'gru1.bias_hh_l0',
              'linear1.weight', 'linear1.bias', 'linear2.weight', 'linear2.bias']:
        sd[k] = torch.from_numpy(w[k])
    net.load_state_dict(sd)
    nets.append(net.to(dev))
erb = torch.tensor(aec_amd.erb_matrix(), dtype=torch.float32, device=dev)
mic, ref, near = (torch.from_numpy(x).to(dev) for x in synth.batch(B, n, seed0=0))
lens = [n] * B
streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(a.inflight - 1)]
side = torch.cuda.Stream(dev) if a.lookahead else None
kstep = [0]


done_ev = {}
tokens = {}


def step(ev=None):
    n = kstep[0]
    k = n % a.inflight
    kstep[0] += 1
    if side is not None:
        gate = done_ev.pop(n - a.inflight + a.lookahead - 1, None)
        if gate is not None and a.paced:
            side.wait_event(gate)
        with torch.cuda.stream(side):
            tokens[n + a.lookahead] = nets[(k + a.lookahead) % a.inflight].prepare_ragged(mic, ref, near, lens)
    with torch.cuda.stream(streams[k]):
        nets[k].forward_ragged(mic, ref, near, erb, lens, lookahead=tokens.pop(n, None))
        if ev is not None:
            ev.record(streams[k])
        e = torch.cuda.Event()
        e.record(streams[k])
        done_ev[n] = e


with torch.no_grad():
    for _ in range(max(a.warmup, a.inflight, a.lookahead)):
        step()
    torch.cuda.synchronize(dev)
    start = torch.cuda.Event(enable_timing=True)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    host = []
    t0 = time.perf_counter()
    start.record(streams[0])
    for i in range(a.steps):
        step(evs[i])
        host.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) * 1e3
done = [start.elapsed_time(e) for e in evs]
print(json.dumps(dict(steps=a.steps, inflight=a.inflight, lookahead=a.lookahead, paced=a.paced, wall_ms=round(el, 3),
                      ms_per_step=round(el / a.steps, 4),
                      batch_done_ms=[round(x, 3) for x in done],
                      host_enqueued_ms=[round(x, 3) for x in host])))
