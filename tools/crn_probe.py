#!/usr/bin/env python3
"""GPU probe for the DCCRN path: relative errors per golden case and dtype,
then a timed run of BASELINE config 3's shape (B streams x N samples) with
the per-stage HIP-event breakdown.  Run on the GPU box:

    python tools/crn_probe.py [--B 256] [--N 160000] [--dtype bf16] [--iters 3]
"""
import argparse
import copy
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
sys.path.insert(0, os.path.join(REPO, 'oracle'))
import aec_amd  # noqa: E402
import crn_oracle as C  # noqa: E402

GOLD = os.path.join(REPO, 'tests', 'golden')


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-30)) if b.size else 0.0


def build(version, conf, dtype, wseed):
    net = (aec_amd.dccrn if version == 1 else aec_amd.dccrn2).DCCRN(conf, dtype=dtype).eval()
    sd = net.state_dict()
    for k, v in C.make_weights(conf, version, wseed).items():
        sd[k] = torch.from_numpy(v)
    net.load_state_dict(sd)
    return net.cuda()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--B', type=int, default=256)
    ap.add_argument('--N', type=int, default=160000)
    ap.add_argument('--dtype', default='bf16')
    ap.add_argument('--iters', type=int, default=3)
    ap.add_argument('--skip-golden', action='store_true')
    a = ap.parse_args()
    if not a.skip_golden:
        meta = json.load(open(os.path.join(GOLD, 'crn_meta.json')))
        for name, m in sorted(meta.items()):
            d = np.load(os.path.join(GOLD, f'crn_{name}.npz'))
            conf = copy.deepcopy(aec_amd.net_conf)
            conf.update(m['overrides'])
            for dt in ('f32', 'bf16', 'fp8'):
                net = build(m['version'], conf, dt, m['weight_seed'])
                T = lambda x: torch.as_tensor(x, device='cuda')[None]
                with torch.no_grad():
                    out, spec, mask = net.forward_ragged(T(d['mic']), T(d['far']), [m['n']], want_mask=True)
                torch.cuda.synchronize()
                print(json.dumps(dict(case=name, dtype=dt, wav=rel(out[0].cpu(), d['out_wav']),
                                      spec=rel(spec[0].cpu(), d['out_spec']), mask=rel(mask[0].cpu(), d['mask']))),
                      flush=True)
    # timed run, config 3 shape
    conf = copy.deepcopy(aec_amd.net_conf)
    net = build(2, conf, a.dtype, 1)
    g = torch.Generator(device='cuda').manual_seed(0)
    mic = 0.1 * torch.randn(a.B, a.N, device='cuda', generator=g)
    far = 0.1 * torch.randn(a.B, a.N, device='cuda', generator=g)
    lens = [a.N] * a.B
    h = net._handle(mic.device)
    with torch.no_grad():
        net.forward_ragged(mic, far, lens, want_spec=False)
        torch.cuda.synchronize()
        h.profile_enable(True)
        h.profile_read()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            out, _, _ = net.forward_ragged(mic, far, lens, want_spec=False)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        ms, calls = h.profile_read()
    frames = a.B * (a.N // 256 + 1)
    print(json.dumps(dict(B=a.B, N=a.N, dtype=a.dtype, ms_per_call=dt * 1e3, frames_per_s=frames / dt,
                          stage_ms={k: v / max(calls, 1) for k, v in
                                    zip(['front', 'encoder', 'lstm', 'decoder', 'back'], ms)},
                          finite=bool(torch.isfinite(out).all()),
                          out_sha1=hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:16])), flush=True)


if __name__ == '__main__':
    main()
