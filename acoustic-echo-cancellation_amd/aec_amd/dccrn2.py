"""``DCCRN`` v2 — drop-in for Stage2_lhm/scripts/network/dccrn2.py:10-218.

Construction follows dccrn2.py:12-116 in the same order (so
``torch.manual_seed(s)`` reproduces the reference's init); the forward runs
on the GPU through ``libaec_hip.so`` (see ``aec_amd.crn``).  Needs
``use_clstm`` (the reference's non-clstm branch references attributes it
never defines, dccrn2.py:114-116,160-162).
"""
from __future__ import annotations

import torch.nn as nn

from .crn import (ComplexBatchNorm, ComplexConvTranspose2d, NavieComplexLSTM, _check_fixed, _ConviSTFTBuffers,
                  _ConvSTFTBuffers, _DCCRNBase, _encoder_decoder, _stft_bases)


class DCCRN(_DCCRNBase):
    VERSION = 2

    def __init__(self, config, dtype='f32', nlms=None):
        super().__init__(config, dtype, nlms)
        _check_fixed(config)
        if not config['use_clstm']:
            raise NotImplementedError('dccrn2.DCCRN needs use_clstm=True (dccrn2.py:114-116)')
        self.win_len = config['win_size']
        self.win_inc = config['hop_size']
        self.fft_len = config['win_size']
        self.win_type = config['win_type']
        self.kernel_num = config['conv_channels']
        self.use_cbn = config['use_cbn']
        self.use_clstm = config['use_clstm']
        self.rnn_layers = config['rnn_layers']
        self.rnn_units = config['rnn_units']
        self.masking_mode = config['masking_mode']
        fwd, inv, win = _stft_bases()
        self.stft = _ConvSTFTBuffers(fwd)
        self.istft = _ConviSTFTBuffers(inv, win)
        self.encoder = nn.ModuleList()
        self.decoder = nn.ModuleList()
        _encoder_decoder(self, config, cbn=self.use_cbn)
        hidden_dim = config['hidden_dim']
        ch = self.kernel_num
        rnns = [NavieComplexLSTM(hidden_dim * ch[-1], hidden_dim * ch[-1]) for _ in range(self.rnn_layers)]
        self.enhance = nn.Sequential(*rnns)                  # dccrn2.py:67-78
        for c in range(len(ch) - 1, 0, -1):                  # dccrn2.py:83-111
            if c != 1:
                self.decoder.append(nn.Sequential(
                    ComplexConvTranspose2d(ch[c] * 2, ch[c - 1], config['kernel_size'], config['stride'],
                                           config['padding'], (1, 0)),
                    ComplexBatchNorm(ch[c - 1]) if self.use_cbn else nn.BatchNorm2d(ch[c - 1]),
                    nn.PReLU()))
            else:
                self.decoder.append(nn.Sequential(
                    ComplexConvTranspose2d(ch[c] * 2, 2, config['kernel_size'], config['stride'],
                                           config['padding'], (1, 0))))

    def forward(self, mic, far, near, echo=None):
        """dccrn2.py:118-218 -> (out_spec, out_wav, near_specs)."""
        if mic.dim() == 1:
            mic, far = mic[None], far[None]
            near = near[None] if near is not None else None
        self._check(mic, far)
        B, N = mic.shape
        out_wav, out_spec, _ = self.forward_ragged(mic, far, [N] * B, want_spec=True)
        near_specs = self.spectra(near) if near is not None else None
        return out_spec, out_wav, near_specs
