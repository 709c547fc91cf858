"""PyTorch-CPU restatement of the reference hot path — TEST / BASELINE ONLY.

Used as ``bench.py``'s ``cpu_baseline`` ("port") and pinned against the
reference goldens by tests/test_oracle_golden.py::test_torch_port_matches_golden.
It keeps the reference's CPU op mix: the STFT as ``conv1d``
with the 514x512 windowed-DFT basis (attention_ccrn.py:45-52), ``nn.GRU``
(ERB.py:293), dense ERB matmuls (ERB.py:282-307) and the iSTFT as two
``conv_transpose1d`` (attention_ccrn.py:82-101) — so its timing represents what
the reference costs on the same host — but normalises each row by its own
mean/std (the drop-in batch=1 semantics).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

WIN, HOP = 512, 256


def bases():
    """(forward basis [514,1,512], inverse basis [514,1,512], window [1,512,1])."""
    n = np.arange(WIN)
    win = 0.5 - 0.5 * np.cos(2 * np.pi * n / WIN)
    k = np.arange(WIN // 2 + 1)[:, None]
    ang = 2 * np.pi * k * n[None] / WIN
    fwd = np.concatenate([np.cos(ang), -np.sin(ang)], 0)
    ck = np.full((WIN // 2 + 1, 1), 2.0)
    ck[0] = ck[-1] = 1.0
    inv = np.concatenate([np.cos(ang) * ck, -np.sin(ang) * ck], 0) / WIN
    inv[WIN // 2 + 1] = 0.0
    inv[-1] = 0.0
    t = lambda a: torch.from_numpy((a * win).astype(np.float32))[:, None, :]
    return t(fwd), t(inv), torch.from_numpy(win.astype(np.float32))[None, :, None]


class TorchPort:
    def __init__(self, weights: dict, erb: np.ndarray):
        self.fwd, self.inv, self.win = bases()
        self.erb = torch.tensor(np.asarray(erb), dtype=torch.float32)
        self.gru = torch.nn.GRU(64, 32, batch_first=True)
        with torch.no_grad():
            for k in ['weight_ih_l0', 'weight_hh_l0', 'bias_ih_l0', 'bias_hh_l0']:
                getattr(self.gru, k).copy_(torch.from_numpy(np.asarray(weights['gru1.' + k])))
        g = lambda k: torch.from_numpy(np.asarray(weights[k], np.float32))
        self.w1, self.b1 = g('linear1.weight'), g('linear1.bias')
        self.w2, self.b2 = g('linear2.weight'), g('linear2.bias')
        self.eye = torch.eye(WIN)[:, None, :]

    def _stft(self, x):
        return F.conv1d(F.pad(x[:, None], [WIN - HOP, WIN - HOP]), self.fwd, stride=HOP)

    @torch.no_grad()
    def __call__(self, mic, ref, near):
        """[B, N] float32 tensors -> (out [B, 256*(N//256)], per-row loss [B])."""
        norm = lambda x: x - (x.mean(1, keepdim=True) / x.std(1, keepdim=True))
        mic, ref, near = norm(mic), norm(ref), norm(near)
        K = WIN // 2 + 1
        S = [self._stft(x) for x in (mic, ref, near)]
        mag = [torch.sqrt(s[:, :K] ** 2 + s[:, K:] ** 2 + 1e-9).transpose(1, 2) for s in S]
        mic_erb, ref_erb, near_erb = (m @ self.erb for m in mag)
        h, _ = self.gru(torch.cat([mic_erb, (mic_erb - ref_erb).abs()], 2))
        o = torch.relu(torch.cat([h, mic_erb], 2) @ self.w1.T + self.b1)
        est = torch.sigmoid(o @ self.w2.T + self.b2) * mic_erb
        gain = (est @ self.erb.T).transpose(1, 2)
        spec = torch.cat([gain * S[0][:, :K], gain * S[0][:, K:]], 1)
        T = spec.shape[-1]
        y = F.conv_transpose1d(spec, self.inv, stride=HOP)
        coff = F.conv_transpose1d(self.win.repeat(1, 1, T) ** 2, self.eye, stride=HOP)
        y = (y / (coff + 1e-8))[..., WIN - HOP:-(WIN - HOP)]
        out = y[:, 0] + 1e-9
        loss = ((near_erb ** 0.5 - est ** 0.5) ** 2).sum((1, 2)) / (T * self.erb.shape[1])
        return out, loss


class TorchTrainPort(TorchPort):
    """One training iteration of scripts/train1.py:199-218 with the reference's
    CPU op mix and autograd: batch-GLOBAL normaliser (ERB.py:254-256 over the
    padded [B, N] batch), batch-summed loss, loss.backward(), torch Adam.
    Baseline / test only (bench.py's training CPU figure)."""

    def __init__(self, weights: dict, erb: np.ndarray, lr=1e-5):
        super().__init__(weights, erb)
        for t in (self.w1, self.b1, self.w2, self.b2):
            t.requires_grad_(True)
        self.params = [self.gru.weight_ih_l0, self.gru.weight_hh_l0, self.gru.bias_ih_l0, self.gru.bias_hh_l0,
                       self.w1, self.b1, self.w2, self.b2]
        self.opt = torch.optim.Adam(self.params, lr=lr)

    def loss(self, mic, ref, near):
        norm = lambda x: x - (x.mean() / x.std())
        mic, ref, near = norm(mic), norm(ref), norm(near)
        K = WIN // 2 + 1
        S = [self._stft(x) for x in (mic, ref, near)]
        mag = [torch.sqrt(s[:, :K] ** 2 + s[:, K:] ** 2 + 1e-9).transpose(1, 2) for s in S]
        mic_erb, ref_erb, near_erb = (m @ self.erb for m in mag)
        h, _ = self.gru(torch.cat([mic_erb, (mic_erb - ref_erb).abs()], 2))
        o = torch.relu(torch.cat([h, mic_erb], 2) @ self.w1.T + self.b1)
        est = torch.sigmoid(o @ self.w2.T + self.b2) * mic_erb
        gain = (est @ self.erb.T).transpose(1, 2)
        spec = torch.cat([gain * S[0][:, :K], gain * S[0][:, K:]], 1)
        T = spec.shape[-1]
        F.conv_transpose1d(spec, self.inv, stride=HOP)          # out_wav, computed (and unused) as in train1.py
        return ((near_erb ** 0.5 - est ** 0.5) ** 2).sum() / (T * self.erb.shape[1])

    def step(self, mic, ref, near):
        self.opt.zero_grad()
        with torch.enable_grad():
            loss = self.loss(mic, ref, near)
        loss.backward()
        self.opt.step()
        return float(loss.detach())
