#!/usr/bin/env python3
"""Where the fused per-hop kernels (crn_stream.hip) differ from the separate
launches: the C5 step at AEC_CRN_STREAM_FUSE = 0 / 1 (front) / 2 (back) / 3,
37 streams x 14 hops, max abs difference and the hops it appears in."""
import os, sys, copy, json
import numpy as np, torch
sys.path.insert(0, 'acoustic-echo-cancellation_amd'); sys.path.insert(0, 'oracle'); sys.path.insert(0,'tests')
import aec_amd, crn_oracle as C
from aec_amd import synth
META = json.load(open('tests/golden/crn_meta.json'))
m = META['v2E_16000']
conf = copy.deepcopy(aec_amd.net_conf)
net = aec_amd.dccrn2.DCCRN(conf, dtype='bf16', nlms=None).eval()
sd = net.state_dict()
for k, v in C.make_weights(conf, 2, m['weight_seed']).items(): sd[k] = torch.from_numpy(v)
net.load_state_dict(sd, strict=True); net = net.to('cuda:0')
B, n = 37, 3328
sig = [synth.scene(n, 2900 + b) for b in range(B)]
nh = n // 256 + 1
M = torch.zeros(B, 256 * (nh + 1), device='cuda:0'); F = torch.zeros_like(M)
M[:, :n] = torch.from_numpy(np.stack([s[0] for s in sig])).cuda(); F[:, :n] = torch.from_numpy(np.stack([s[1] for s in sig])).cuda()
res = {}
for flag in ('0', '1', '2', '3'):
    os.environ['AEC_CRN_STREAM_FUSE'] = flag
    net.stream_open(B)
    with torch.no_grad():
        outs = [net.stream_step(M[:, 256 * k:256 * (k + 1)], F[:, 256 * k:256 * (k + 1)]).clone() for k in range(nh)]
    torch.cuda.synchronize()
    res[flag] = torch.stack(outs, 1).cpu().numpy()   # [B, hop, 256]
for f in '123':
    d = np.abs(res[f] - res['0'])
    idx = np.argwhere(d > 0)
    print(f, 'max diff', d.max(), 'n diff', len(idx), 'first hops with diff', sorted(set(idx[:, 1].tolist()))[:5] if len(idx) else None,
          'rel', float(np.sqrt((d**2).mean()) / np.sqrt((res['0']**2).mean())))
