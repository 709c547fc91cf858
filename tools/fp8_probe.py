"""MX-fp8 DCCRN probe (run on the GPU box): fp8 vs bf16 error on the golden
cases and the C5 hipGraph streaming step / C3 batch timings.
    python tools/fp8_probe.py"""
import copy
import json
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, 'acoustic-echo-cancellation_amd'), os.path.join(R, 'oracle'), os.path.join(R, 'tests')]
import aec_amd  # noqa: E402
import bench  # noqa: E402
import crn_oracle as C  # noqa: E402

G = os.path.join(R, 'tests', 'golden')
meta = json.load(open(os.path.join(G, 'crn_meta.json')))
res = {}
for name in ['v2E_2125', 'v2E_16000', 'v1_2125']:
    m = meta[name]
    d = np.load(os.path.join(G, f'crn_{name}.npz'))
    for dt in ('bf16', 'fp8'):
        conf = copy.deepcopy(aec_amd.net_conf)
        conf.update(m['overrides'])
        net = (aec_amd.dccrn if m['version'] == 1 else aec_amd.dccrn2).DCCRN(conf, dtype=dt).eval()
        sd = net.state_dict()
        for k, v in C.make_weights(conf, m['version'], m['weight_seed']).items():
            sd[k] = torch.from_numpy(v)
        net.load_state_dict(sd, strict=True)
        net = net.to('cuda:0')
        T = lambda a: torch.as_tensor(np.asarray(a), device='cuda:0')[None]
        with torch.no_grad():
            out, _, mask = net.forward_ragged(T(d['mic']), T(d['far']), [m['n']], want_spec=False, want_mask=True)
        o = out[0].cpu().numpy().astype(np.float64)
        r = d['out_wav'].astype(np.float64)
        res[f'{name}/{dt}/wav_rel_rms'] = float(np.sqrt(np.mean((o - r) ** 2)) / np.sqrt(np.mean(r ** 2)))
print(json.dumps(res, indent=1), flush=True)
dev = torch.device('cuda', 0)
for dt in ('bf16', 'fp8'):
    print(dt, 'c5 stream', json.dumps(bench.run_c5_stream(dev, dtype=dt)), flush=True)
