"""``DCCRN`` v1 — drop-in for Stage2_lhm/scripts/network/dccrn.py:453-594.

Construction follows dccrn.py:454-521 in the same order (so
``torch.manual_seed(s)`` reproduces the reference's init); the forward runs
on the GPU through ``libaec_hip.so`` (see ``aec_amd.crn``).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .crn import (ComplexConvTranspose2d, _check_fixed, _ConviSTFTBuffers, _ConvSTFTBuffers, _DCCRNBase,
                  _encoder_decoder, _stft_bases)


class DCCRN(_DCCRNBase):
    VERSION = 1

    def __init__(self, config, dtype='f32', nlms=None):
        super().__init__(config, dtype, nlms)
        _check_fixed(config)
        ch = config['conv_channels']
        self.encoder = nn.ModuleList()
        self.decoder = nn.ModuleList()
        self.tanh = nn.Tanh()
        _encoder_decoder(self, config, cbn=False)
        for c in range(len(ch) - 1, 0, -1):               # dccrn.py:479-509
            if c != 1:
                self.decoder.append(nn.Sequential(
                    ComplexConvTranspose2d(ch[c] * 2, ch[c - 1], config['kernel_size'], config['stride'],
                                           config['padding'], (1, 0)),
                    nn.BatchNorm2d(ch[c - 1]), nn.PReLU()))
            else:
                self.decoder.append(nn.Sequential(
                    ComplexConvTranspose2d(ch[c] * 2, 2, config['kernel_size'], config['stride'],
                                           config['padding'], (1, 0)),
                    nn.BatchNorm2d(2), nn.Tanh()))
        self.win_type = 'hann'
        self.win_len = config['win_size']
        self.win_inc = config['hop_size']
        self.lstm = nn.LSTM(input_size=ch[-1] * 4, hidden_size=ch[-1] * 4, num_layers=1)   # dccrn.py:514
        fwd, inv, win = _stft_bases()
        self.stft = _ConvSTFTBuffers(fwd)
        self.istft = _ConviSTFTBuffers(inv, win)

    def forward(self, mic, far, near, echo):
        """dccrn.py:532-594 -> (out_wav, out_spec, near_specs, loss)."""
        if mic.dim() == 1:
            mic, far, near, echo = mic[None], far[None], near[None], echo[None]
        self._check(mic, far, near, echo)
        B, N = mic.shape
        out_wav, out_spec, mask = self.forward_ragged(mic, far, [N] * B, want_spec=True, want_mask=True)
        near_specs = self.spectra(near)
        # training loss (dccrn.py:556-581) from the GPU spectra and mask (elementwise)
        # (an NLMS network masks the error spectrum E, so E is the cRM reference)
        ms = self.error_spectra(mic.device) if self.nlms else self.spectra(mic)
        es = self.spectra(echo)
        K = 257
        mr, mi = ms[:, :K], ms[:, K:]
        nr, ni = near_specs[:, :K], near_specs[:, K:]
        er, ei = es[:, :K], es[:, K:]
        den = mr ** 2 + mi ** 2 + 1e-9
        c_r = (mr * nr + mi * ni) / den
        c_i = (mr * ni - mi * nr) / den
        mk_r = torch.nn.functional.pad(mask[:, 0], [0, 0, 1, 0])
        mk_i = torch.nn.functional.pad(mask[:, 1], [0, 0, 1, 0])
        loss_mask = torch.mean((mk_r - c_r) ** 2) + torch.mean((mk_i - c_i) ** 2)
        xr = er * mk_r - ei * mk_i
        xi = er * mk_i + ei * mk_r
        loss = 0.3 * loss_mask + 0.7 * (torch.mean(xr ** 2) + torch.mean(xi ** 2))
        return out_wav, out_spec, near_specs, loss
