#!/usr/bin/env python3
"""CPU estimate of the output error an MX-fp8 LSTM recurrence adds (C5 per-hop
step): the torch DCCRN port (oracle/torch_crn_port.py,
net_conf, v2) with W_hh and h_{t-1} rounded to OCP e4m3 with one E8M0 scale
per 32 k (the device quantiser's rule, crn_api.hip upload_mx8) against the f32
port.  Also rounds the LSTM input projections' operands the same way (the
fp8 path of round 2) so the two error sources can be compared.

    python tools/fp8_rec_sim.py [seconds] [streams]
"""
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, 'oracle'), os.path.join(R, 'acoustic-echo-cancellation_amd')]
import torch_crn_port as P  # noqa: E402
from aec_amd import configs, synth  # noqa: E402


def mx8(x):
    """e4m3 (RNE, saturating) with an E8M0 scale 2^(floor(log2 amax) - 8) per 32 along the last dim."""
    s = x.shape
    g = x.reshape(*s[:-1], s[-1] // 32, 32).double()
    amax = g.abs().amax(-1, keepdim=True)
    e = torch.floor(torch.log2(torch.where(amax > 0, amax, torch.ones_like(amax))))
    scale = torch.where(amax > 0, 2.0 ** (e - 8), torch.ones_like(amax))
    v = (g / scale).clamp(-448, 448)
    a = v.abs()
    E = torch.floor(torch.log2(torch.where(a > 0, a, torch.ones_like(a)))).clamp(min=-6)
    q = torch.round(a / 2.0 ** (E - 3)) * 2.0 ** (E - 3)          # 3 mantissa bits (subnormal step 2^-9)
    return (torch.sign(v) * q.clamp(max=448) * scale).reshape(s).to(x.dtype)


class QLSTM:
    """nn.LSTM(eval) restated per step with optional MX rounding of the recurrent / input operands."""

    def __init__(self, m, rec, inp):
        self.wih, self.whh = m.weight_ih_l0.detach(), m.weight_hh_l0.detach()
        self.b = (m.bias_ih_l0 + m.bias_hh_l0).detach()
        self.rec, self.inp = rec, inp
        if rec:
            self.whh = mx8(self.whh)
        if inp:
            self.wih = mx8(self.wih)

    def __call__(self, x):
        T, B, _ = x.shape
        H = self.whh.shape[1]
        if self.inp:
            x = mx8(x)
        gx = x @ self.wih.T + self.b
        h = torch.zeros(B, H)
        c = torch.zeros(B, H)
        out = []
        for t in range(T):
            hq = mx8(h) if self.rec else h
            g = gx[t] + hq @ self.whh.T
            i, f, gg, o = g.chunk(4, 1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
            h = torch.sigmoid(o) * torch.tanh(c)
            out.append(h)
        return torch.stack(out), None


def main():
    sec = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    torch.set_num_threads(8)
    conf = configs.net_conf
    port = P.fixture_port(conf, 2, 0)
    n = int(sec * 16000)
    mic = np.stack([synth.scene(n, 11 + i)[0] for i in range(B)]).astype(np.float32)
    far = np.stack([synth.scene(n, 11 + i)[1] for i in range(B)]).astype(np.float32)
    mic_t, far_t = torch.from_numpy(mic), torch.from_numpy(far)
    ref = port(mic_t, far_t)
    base = dict(port.lstms)
    rel = lambda y: float(torch.sqrt(torch.mean((y - ref) ** 2) / torch.mean(ref ** 2)))
    for name, rec, inp in (('exact restated', False, False), ('input MX', False, True),
                           ('recurrent MX', True, False), ('input + recurrent MX', True, True)):
        port.lstms = {k: QLSTM(m, rec, inp) for k, m in base.items()}
        print(f'{name:22s} out_wav rel RMS vs f32: {rel(port(mic_t, far_t)):.5f}', flush=True)


if __name__ == '__main__':
    main()
