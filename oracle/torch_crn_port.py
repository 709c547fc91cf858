"""PyTorch-CPU restatement of the DCCRN eval forward — TEST / BASELINE
INFRASTRUCTURE ONLY (imported by tests/ and bench.py's cpu_baseline leg).

Same op mix as the reference (Stage2_lhm/scripts/network/dccrn.py:453-594,
dccrn2.py:10-218): conv1d DFT-basis STFT, per-layer F.conv2d /
F.conv_transpose2d on real/imag halves (ComplexConv2d, dccrn.py:140-153 /
:194-207), eval (Complex)BatchNorm, PReLU, nn.LSTM (real and complex
NavieComplexLSTM, dccrn.py:423-450), masks, conv_transpose1d iSTFT.  Float32
on host cores; pinned against the reference goldens by
tests/test_crn_oracle.py.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

import crn_oracle as C
from aec_oracle import hann


def _bases():
    n = np.arange(512)
    k = np.arange(257)[:, None]
    win = hann()
    ang = 2 * np.pi * k * n[None, :] / 512
    fwd = np.concatenate([np.cos(ang), -np.sin(ang)], 0) * win
    ck = np.full((257, 1), 2.0)
    ck[0] = ck[-1] = 1.0
    inv = np.concatenate([np.cos(ang) * ck, -np.sin(ang) * ck], 0) / 512
    inv[257] = 0.0
    inv[-1] = 0.0
    inv = inv * win
    t = lambda a: torch.from_numpy(a.astype(np.float32))[:, None, :]
    return t(fwd), t(inv), torch.from_numpy(win.astype(np.float32))


class TorchCrnPort:
    """nlms: None (the reference network) or dict(taps, mu, beta, delta): the
    build-defined FD-NLMS front end of include/aec_crn.h, restated as in
    crn_oracle.forward(..., nlms=...) — the mic spectrum is replaced (encoder
    input and masking) by the a-priori error of aec_oracle.nlms (float64)
    driven by the far spectrum."""

    def __init__(self, w, conf, version, nlms=None):
        self.conf, self.version, self.nlms = conf, version, nlms
        self.w = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in w.items()}
        self.fwd, self.inv, self.win = _bases()
        self.cbn = version == 2 and conf['use_cbn']
        self.lstms = {}
        if version == 1:
            self.lstms['lstm'] = self._lstm('lstm')
        else:
            for l in range(conf['rnn_layers']):
                for part in ('real_lstm', 'imag_lstm'):
                    self.lstms[f'enhance.{l}.{part}'] = self._lstm(f'enhance.{l}.{part}')

    def _lstm(self, p):
        wih = self.w[f'{p}.weight_ih_l0']
        m = torch.nn.LSTM(wih.shape[1], wih.shape[0] // 4)
        with torch.no_grad():
            m.weight_ih_l0.copy_(wih)
            m.weight_hh_l0.copy_(self.w[f'{p}.weight_hh_l0'])
            m.bias_ih_l0.copy_(self.w[f'{p}.bias_ih_l0'])
            m.bias_hh_l0.copy_(self.w[f'{p}.bias_hh_l0'])
        return m.eval()

    def stft(self, x):                                           # dccrn.py:45-52
        return F.conv1d(F.pad(x[:, None], [256, 256]), self.fwd, stride=256)

    def istft(self, spec):                                       # dccrn.py:80-100
        out = F.conv_transpose1d(spec, self.inv, stride=256)
        t = (self.win[None, :, None] ** 2).repeat(1, 1, spec.shape[-1])
        coff = F.conv_transpose1d(t, torch.eye(512)[:, None, :], stride=256)
        return (out / (coff + 1e-8))[..., 256:-256][:, 0]

    def _cconv(self, x, p, transposed):
        c = x.shape[1] // 2
        xr, xi = x[:, :c], x[:, c:]
        op = (lambda z, w, b: F.conv_transpose2d(z, w, b, stride=(2, 1), padding=(2, 0), output_padding=(1, 0))) \
            if transposed else (lambda z, w, b: F.conv2d(z, w, b, stride=(2, 1), padding=(2, 0)))
        R = lambda z: op(z, self.w[f'{p}.real_conv.weight'], self.w[f'{p}.real_conv.bias'])
        I = lambda z: op(z, self.w[f'{p}.imag_conv.weight'], self.w[f'{p}.imag_conv.bias'])
        return torch.cat([R(xr) - I(xi), I(xr) + R(xi)], 1)

    def _norm(self, x, p, cbn):
        if not cbn:
            g = lambda n: self.w[f'{p}.{n}'][None, :, None, None]
            return (x - g('running_mean')) / torch.sqrt(g('running_var') + 1e-5) * g('weight') + g('bias')
        c = x.shape[1] // 2
        g = lambda n: self.w[f'{p}.{n}'][None, :, None, None]
        xr, xi = x[:, :c] - g('RMr'), x[:, c:] - g('RMi')
        Vrr, Vri, Vii = g('RVrr') + 1e-5, g('RVri'), g('RVii') + 1e-5
        s = torch.sqrt(Vrr * Vii - Vri * Vri)
        t = torch.sqrt(Vrr + Vii + 2 * s)
        rst = 1.0 / (s * t)
        Urr, Uii, Uri = (s + Vii) * rst, (s + Vrr) * rst, -Vri * rst
        Wrr, Wri, Wii = g('Wrr'), g('Wri'), g('Wii')
        Zrr, Zri = Wrr * Urr + Wri * Uri, Wrr * Uri + Wri * Uii
        Zir, Zii = Wri * Urr + Wii * Uri, Wri * Uri + Wii * Uii
        return torch.cat([Zrr * xr + Zri * xi + g('Br'), Zir * xr + Zii * xi + g('Bi')], 1)

    @torch.no_grad()
    def __call__(self, mic, far):
        """mic/far [B, N] float32 (CPU) -> out_wav [B, 256*(N//256)]."""
        L = len(self.conf['conv_channels']) - 1
        ms, fs = self.stft(mic), self.stft(far)
        mr, mi, fr, fi = ms[:, :257], ms[:, 257:], fs[:, :257], fs[:, 257:]
        if self.nlms:
            from aec_oracle import nlms as _nlms
            nl = self.nlms
            E = [_nlms((mr[b].double() + 1j * mi[b].double()).numpy().T, (fr[b].double() + 1j * fi[b].double()).numpy().T,
                       taps=nl.get('taps', 4), mu=nl.get('mu', 0.3), beta=nl.get('beta', 0.5),
                       delta=nl.get('delta', 1e-4)).T for b in range(mr.shape[0])]
            mr = torch.from_numpy(np.stack([e.real for e in E]).astype(np.float32))
            mi = torch.from_numpy(np.stack([e.imag for e in E]).astype(np.float32))
        out = torch.stack([mr, fr, mi, fi], 1)[:, :, 1:]
        skips = []
        for i in range(L):
            out = self._cconv(out, f'encoder.{i}.0', False)
            out = F.prelu(self._norm(out, f'encoder.{i}.1', self.cbn), self.w[f'encoder.{i}.2.weight'])
            skips.append(out)
        B, Cc, D, T = out.shape
        out = out.permute(3, 0, 1, 2)
        if self.version == 1:
            y, _ = self.lstms['lstm'](out.reshape(T, B, Cc * D))
            out = y.reshape(T, B, Cc, D)
        else:
            xr = out[:, :, :Cc // 2].reshape(T, B, -1)
            xi = out[:, :, Cc // 2:].reshape(T, B, -1)
            for l in range(self.conf['rnn_layers']):
                R, I = self.lstms[f'enhance.{l}.real_lstm'], self.lstms[f'enhance.{l}.imag_lstm']
                rr, ri, ir, ii = R(xr)[0], I(xr)[0], R(xi)[0], I(xi)[0]
                xr, xi = rr - ii, ir + ri
            out = torch.cat([xr.reshape(T, B, Cc // 2, D), xi.reshape(T, B, Cc // 2, D)], 2)
        out = out.permute(1, 2, 3, 0)
        for d in range(L):
            a, b = out, skips[-1 - d]
            ca, cb = a.shape[1] // 2, b.shape[1] // 2
            out = torch.cat([a[:, :ca], b[:, :cb], a[:, ca:], b[:, cb:]], 1)
            out = self._cconv(out, f'decoder.{d}.0', True)
            if d != L - 1:
                out = F.prelu(self._norm(out, f'decoder.{d}.1', self.cbn), self.w[f'decoder.{d}.2.weight'])
            elif self.version == 1:
                out = torch.tanh(self._norm(out, f'decoder.{d}.1', False))
        mkr, mki = F.pad(out[:, 0], [0, 0, 1, 0]), F.pad(out[:, 1], [0, 0, 1, 0])
        mode = 'C' if self.version == 1 else self.conf['masking_mode']
        if mode == 'E':
            mags = torch.sqrt(mr ** 2 + mi ** 2 + 1e-8)
            ph = torch.atan2(mi, mr)
            mm = torch.sqrt(mkr ** 2 + mki ** 2)
            mph = torch.atan2(mki / (mm + 1e-8), mkr / (mm + 1e-8))
            em = torch.tanh(mm) * mags
            er, ei = em * torch.cos(ph + mph), em * torch.sin(ph + mph)
        elif mode == 'C':
            er, ei = mr * mkr - mi * mki, mr * mki + mi * mkr
        else:
            er, ei = mr * mkr, mi * mki
        return self.istft(torch.cat([er, ei], 1))


def fixture_port(conf, version, seed):
    return TorchCrnPort(C.make_weights(conf, version, seed), conf, version)


class TorchCrnStreamPort(TorchCrnPort):
    """The same op mix stepped one 256-sample hop per stream per call — the
    CPU counterpart of aec_crn_stream_step (BASELINE config 5), used as the
    c5_stream_fp8 cpu_baseline in bench.py.  Frame s = [hop s-1, hop s]; the
    encoder / decoder convs have time extent 1, so a frame goes through them
    alone; the LSTM state (h, c) of each NavieComplexLSTM cell x input sequence
    is carried per stream, the FD-NLMS state (taps, far history, power) per
    stream and bin, and the iSTFT overlap-adds the previous frame's second
    half: step s emits hop s-1 of __call__'s out_wav."""

    def stream_open(self, B):
        L = len(self.conf['conv_channels']) - 1
        self.B = B
        self.prev = torch.zeros(2, B, 256)
        self.tail = torch.zeros(B, 1, 256)
        self.state = {}
        if self.nlms:
            t = self.nlms.get('taps', 4)
            self.nW = torch.zeros(B, t, 257, dtype=torch.complex128)
            self.nH = torch.zeros(B, t, 257, dtype=torch.complex128)
            self.nP = torch.zeros(B, 257, dtype=torch.float64)
        w2 = self.win ** 2
        self.coff = (w2[:256] + w2[256:] + 1e-8)[None, None]
        self.L = L

    def _lstm_step(self, key, x):
        y, self.state[key] = self.lstms[key[0]](x[None], self.state.get(key))
        return y[0]

    @torch.no_grad()
    def step(self, mic_hop, far_hop):
        """mic_hop / far_hop [B, 256] float32 -> out hop [B, 256]."""
        frames = torch.stack([torch.cat([self.prev[0], mic_hop], 1), torch.cat([self.prev[1], far_hop], 1)])
        self.prev = torch.stack([mic_hop, far_hop])
        s = F.conv1d(frames.reshape(-1, 1, 512), self.fwd)[..., 0].reshape(2, self.B, 514)
        mr, mi, fr, fi = s[0, :, :257], s[0, :, 257:], s[1, :, :257], s[1, :, 257:]
        if self.nlms:
            nl = self.nlms
            D = torch.complex(mr.double(), mi.double())
            self.nH = torch.roll(self.nH, 1, dims=1)
            self.nH[:, 0] = torch.complex(fr.double(), fi.double())
            e = D - (self.nW * self.nH).sum(1)
            beta = nl.get('beta', 0.5)
            self.nP = beta * self.nP + (1 - beta) * (self.nH.abs() ** 2).sum(1)
            self.nW = self.nW + nl.get('mu', 0.3) * e[:, None] * self.nH.conj() / (self.nP + nl.get('delta', 1e-4))[:, None]
            mr, mi = e.real.float(), e.imag.float()
        out = torch.stack([mr, fr, mi, fi], 1)[:, :, 1:, None]
        skips = []
        for i in range(self.L):
            out = self._cconv(out, f'encoder.{i}.0', False)
            out = F.prelu(self._norm(out, f'encoder.{i}.1', self.cbn), self.w[f'encoder.{i}.2.weight'])
            skips.append(out)
        B, Cc, D, _ = out.shape
        if self.version == 1:
            out = self._lstm_step(('lstm', 0), out.reshape(B, Cc * D)).reshape(B, Cc, D, 1)
        else:
            xr, xi = out[:, :Cc // 2].reshape(B, -1), out[:, Cc // 2:].reshape(B, -1)
            for l in range(self.conf['rnn_layers']):
                Rk, Ik = f'enhance.{l}.real_lstm', f'enhance.{l}.imag_lstm'
                rr, ri = self._lstm_step((Rk, 'r'), xr), self._lstm_step((Ik, 'r'), xr)
                ir, ii = self._lstm_step((Rk, 'i'), xi), self._lstm_step((Ik, 'i'), xi)
                xr, xi = rr - ii, ir + ri
            out = torch.cat([xr.reshape(B, Cc // 2, D), xi.reshape(B, Cc // 2, D)], 1)[..., None]
        for d in range(self.L):
            a, b = out, skips[-1 - d]
            ca, cb = a.shape[1] // 2, b.shape[1] // 2
            out = torch.cat([a[:, :ca], b[:, :cb], a[:, ca:], b[:, cb:]], 1)
            out = self._cconv(out, f'decoder.{d}.0', True)
            if d != self.L - 1:
                out = F.prelu(self._norm(out, f'decoder.{d}.1', self.cbn), self.w[f'decoder.{d}.2.weight'])
            elif self.version == 1:
                out = torch.tanh(self._norm(out, f'decoder.{d}.1', False))
        mkr, mki = F.pad(out[:, 0, :, 0], [1, 0]), F.pad(out[:, 1, :, 0], [1, 0])
        mode = 'C' if self.version == 1 else self.conf['masking_mode']
        if mode == 'E':
            mags = torch.sqrt(mr ** 2 + mi ** 2 + 1e-8)
            ph = torch.atan2(mi, mr)
            mm = torch.sqrt(mkr ** 2 + mki ** 2)
            mph = torch.atan2(mki / (mm + 1e-8), mkr / (mm + 1e-8))
            em = torch.tanh(mm) * mags
            er, ei = em * torch.cos(ph + mph), em * torch.sin(ph + mph)
        elif mode == 'C':
            er, ei = mr * mkr - mi * mki, mr * mki + mi * mkr
        else:
            er, ei = mr * mkr, mi * mki
        y = F.conv_transpose1d(torch.cat([er, ei], 1)[..., None], self.inv)     # [B, 1, 512]
        hop = (self.tail + y[..., :256]) / self.coff
        self.tail = y[..., 256:]
        return hop[:, 0]
