#!/usr/bin/env python3
"""C5 per-hop step in one launch mode, for a tracer:
  C5_GRAPH=0|1 STREAMS=256 HOPS=200 python tools/c5_mode_prof.py
256 streams (NLMS -> DCCRN fp8, net_conf), 60 untimed hops, then HOPS hops
back to back; prints ms per hop and the library's hop counters."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
import torch  # noqa: E402
import aec_amd  # noqa: E402

graph = os.environ.get('C5_GRAPH', '0') == '1'
side = os.environ.get('C5_SIDE', '0') == '1'          # step on a created (non-default) torch stream
B = int(os.environ.get('STREAMS', '256'))
hops = int(os.environ.get('HOPS', '200'))
dev = torch.device('cuda', 0)
torch.manual_seed(0)
net = aec_amd.dccrn2.DCCRN(dict(aec_amd.net_conf), dtype='fp8', nlms=aec_amd.nlms_conf).eval().to(dev)
net.stream_open(B, device=dev, graph=graph)
if side:
    torch.cuda.set_stream(torch.cuda.Stream(dev))
g = torch.Generator(device=dev).manual_seed(5)
mic = 0.1 * torch.randn(B, 256, device=dev, generator=g)
far = 0.1 * torch.randn(B, 256, device=dev, generator=g)
out = torch.empty(B, 256, device=dev)
with torch.no_grad():
    for _ in range(60):
        net.stream_step(mic, far, out)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(hops):
        net.stream_step(mic, far, out)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
print(json.dumps(dict(graph=graph, side_stream=side, streams=B, hops=hops, ms_per_hop=round(el / hops * 1e3, 4), stats=net.stream_stats())))
