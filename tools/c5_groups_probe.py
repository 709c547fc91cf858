#!/usr/bin/env python3
"""C5 per-hop step with the 256 streams split into G groups in flight: G handles
(same weights) of 256 / G streams each, stepped on G HIP streams (one hop of
every stream per step, as the single handle).  The kernels of a hop are latency
chains that leave CUs idle; independent groups overlap them.
  python tools/c5_groups_probe.py [--groups 1,2,4] [--hops 200] [--graph 0,1]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
import torch  # noqa: E402
import aec_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--groups', default='1,2,4')
ap.add_argument('--graph', default='0,1')
ap.add_argument('--hops', type=int, default=200)
ap.add_argument('--streams', type=int, default=256)
ap.add_argument('--rounds', type=int, default=2)
a = ap.parse_args()
dev = torch.device('cuda', 0)
torch.manual_seed(0)
conf = dict(aec_amd.net_conf)
base = aec_amd.dccrn2.DCCRN(conf, dtype='fp8', nlms=aec_amd.nlms_conf).eval().to(dev)
nets = [base]
B = a.streams
g = torch.Generator(device=dev).manual_seed(5)
mic = 0.1 * torch.randn(B, 256, device=dev, generator=g)
far = 0.1 * torch.randn(B, 256, device=dev, generator=g)
out = torch.empty(B, 256, device=dev)


def run(G, graph, hops):
    while len(nets) < G:
        n2 = aec_amd.dccrn2.DCCRN(conf, dtype='fp8', nlms=aec_amd.nlms_conf).eval()
        n2.load_state_dict(base.state_dict())
        nets.append(n2.to(dev))
    bs = B // G
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(G - 1)]
    for i in range(G):
        nets[i].stream_open(bs, device=dev, graph=bool(graph))
    cur = torch.cuda.current_stream(dev)

    def hop():
        for i in range(G):
            with torch.cuda.stream(streams[i]):
                nets[i].stream_step(mic[i * bs:(i + 1) * bs], far[i * bs:(i + 1) * bs], out[i * bs:(i + 1) * bs])

    with torch.no_grad():
        tw = time.perf_counter()
        while (time.perf_counter() - tw) < 0.05:
            for _ in range(10):
                hop()
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(hops):
            hop()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
    return el / hops * 1e3


res = []
for r in range(a.rounds):
    for graph in [int(x) for x in a.graph.split(',')]:
        for G in [int(x) for x in a.groups.split(',')]:
            ms = run(G, graph, a.hops)
            res.append(dict(round=r, groups=G, graph=graph, ms_per_hop=round(ms, 4), frames_per_s=round(B / ms * 1e3, 1)))
            print(json.dumps(res[-1]), flush=True)
