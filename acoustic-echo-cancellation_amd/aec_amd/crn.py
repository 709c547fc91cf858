"""DCCRN (complex CRN) drop-ins — the gfx950 path of the reference's two CRNs.

Reference: ``DCCRN`` in Stage2_lhm/scripts/network/dccrn.py:453-594 ("v1")
and ``DCCRN`` in Stage2_lhm/scripts/network/dccrn2.py:10-218 ("v2"), plus
their layers (ComplexConv2d / ComplexConvTranspose2d / ComplexBatchNorm /
NavieComplexLSTM, dccrn.py:103-450).

Same constructor ``DCCRN(config)`` (the ``configs.net_conf`` dict,
configs.py:29-46), same submodule / parameter / buffer names (the reference
``state_dict`` loads strictly), the reference's init in the reference's RNG
order, and the same ``forward(mic, far, near, echo)`` outputs:

* v1: ``(out_wav, out_spec, near_specs, loss)`` (dccrn.py:532-594);
* v2: ``(out_spec, out_wav, near_specs)`` (dccrn2.py:118-218).

Eval-mode inference only (BatchNorm running statistics, as
``net.eval()``); it raises in training mode or under autograd.  The whole
network runs in ``libaec_hip.so`` (include/aec_crn.h): ``dtype='f32'``
(exact f32 MFMA, the parity path), ``dtype='bf16'`` (bf16 MFMA with f32
accumulation, the throughput path of BASELINE config 3) or ``dtype='fp8'``
(bf16, with the LSTM input projections -- half the weights -- as MX-fp8:
OCP e4m3 weights and activations with an E8M0 scale per 32 k on the gfx950
scaled MFMA; BASELINE config 5).  No CPU fallback.

Rows of a [B, N] batch are independent in eval mode (nothing couples
utterances), so batching is exact; ``forward_ragged`` takes per-row lengths.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .little_net import HOP, _ConviSTFTBuffers, _ConvSTFTBuffers, _stft_bases


# --------------------------------------------------------------------------
# parameter holders with the reference's names and init (dccrn.py:103-450)
# --------------------------------------------------------------------------
class ComplexConv2d(nn.Module):
    """dccrn.py:103-153 (init :135-138)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, dilation=1, groups=1):
        super().__init__()
        self.real_conv = nn.Conv2d(in_channels // 2, out_channels // 2, kernel_size, stride, padding=padding,
                                   dilation=dilation, groups=groups)
        self.imag_conv = nn.Conv2d(in_channels // 2, out_channels // 2, kernel_size, stride, padding=padding,
                                   dilation=dilation, groups=groups)
        nn.init.normal_(self.real_conv.weight.data, std=0.05)
        nn.init.normal_(self.imag_conv.weight.data, std=0.05)
        nn.init.constant_(self.real_conv.bias, 0.)
        nn.init.constant_(self.imag_conv.bias, 0.)


class ComplexConvTranspose2d(nn.Module):
    """dccrn.py:156-207 (init :178-181)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, output_padding):
        super().__init__()
        self.real_conv = nn.ConvTranspose2d(in_channels // 2, out_channels // 2, kernel_size, stride,
                                            padding=padding, output_padding=output_padding)
        self.imag_conv = nn.ConvTranspose2d(in_channels // 2, out_channels // 2, kernel_size, stride,
                                            padding=padding, output_padding=output_padding)
        nn.init.normal_(self.real_conv.weight, std=0.05)
        nn.init.normal_(self.imag_conv.weight, std=0.05)
        nn.init.constant_(self.real_conv.bias, 0.)
        nn.init.constant_(self.imag_conv.bias, 0.)


class ComplexBatchNorm(nn.Module):
    """dccrn.py:210-253: affine 2x2 W, bias, running mean / covariance."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1):
        super().__init__()
        c = num_features // 2
        self.num_features, self.eps, self.momentum = c, eps, momentum
        self.Wrr = nn.Parameter(torch.Tensor(c))
        self.Wri = nn.Parameter(torch.Tensor(c))
        self.Wii = nn.Parameter(torch.Tensor(c))
        self.Br = nn.Parameter(torch.Tensor(c))
        self.Bi = nn.Parameter(torch.Tensor(c))
        self.register_buffer('RMr', torch.zeros(c))
        self.register_buffer('RMi', torch.zeros(c))
        self.register_buffer('RVrr', torch.ones(c))
        self.register_buffer('RVri', torch.zeros(c))
        self.register_buffer('RVii', torch.ones(c))
        self.register_buffer('num_batches_tracked', torch.tensor(0, dtype=torch.long))
        self.Br.data.zero_()
        self.Bi.data.zero_()
        self.Wrr.data.fill_(1)
        self.Wri.data.uniform_(-.9, +.9)
        self.Wii.data.fill_(1)


class NavieComplexLSTM(nn.Module):
    """dccrn.py:423-450: real_lstm / imag_lstm over input_size // 2."""

    def __init__(self, input_size, hidden_size, bidirectional=False, batch_first=False):
        super().__init__()
        if bidirectional:
            raise NotImplementedError('bidirectional NavieComplexLSTM (dccrn2.py uses bidirectional=False)')
        self.input_dim = input_size // 2
        self.rnn_units = hidden_size // 2
        self.real_lstm = nn.LSTM(self.input_dim, self.rnn_units, num_layers=1, batch_first=False)
        self.imag_lstm = nn.LSTM(self.input_dim, self.rnn_units, num_layers=1, batch_first=False)


class _DCCRNBase(nn.Module):
    VERSION = 0

    def __init__(self, config, dtype='f32', nlms=None):
        super().__init__()
        self.config = config
        self.dtype_name = dtype
        self.nlms = dict(nlms) if nlms else None   # build-defined FD-NLMS front end (include/aec_crn.h)
        self._handles = {}
        self._p_key = {}
        self._last_shape = {}                      # device index -> (B, Tmax) of the last forward

    # ---- parameter blob (include/aec_crn.h order) ---------------------------
    def _norm_names(self, prefix, cbn):
        if cbn:
            return [f'{prefix}.{n}' for n in ('Wrr', 'Wri', 'Wii', 'Br', 'Bi', 'RMr', 'RMi', 'RVrr', 'RVri', 'RVii')]
        return [f'{prefix}.{n}' for n in ('weight', 'bias', 'running_mean', 'running_var')]

    def param_names(self):
        ch = list(self.config['conv_channels'])
        L = len(ch) - 1
        cbn = self.VERSION == 2 and self.config['use_cbn']
        conv = lambda p: [f'{p}.{c}.{w}' for c in ('real_conv', 'imag_conv') for w in ('weight', 'bias')]
        names = []
        for i in range(L):
            names += conv(f'encoder.{i}.0') + self._norm_names(f'encoder.{i}.1', cbn) + [f'encoder.{i}.2.weight']
        for d in range(L):
            names += conv(f'decoder.{d}.0')
            if d != L - 1:
                names += self._norm_names(f'decoder.{d}.1', cbn) + [f'decoder.{d}.2.weight']
            elif self.VERSION == 1:
                names += self._norm_names(f'decoder.{d}.1', False)
        lstm = lambda p: [f'{p}.{w}' for w in ('weight_ih_l0', 'weight_hh_l0', 'bias_ih_l0', 'bias_hh_l0')]
        if self.VERSION == 1:
            names += lstm('lstm')
        else:
            for l in range(self.config['rnn_layers']):
                names += lstm(f'enhance.{l}.real_lstm') + lstm(f'enhance.{l}.imag_lstm')
        return names

    def params_blob(self):
        sd = self.state_dict()
        return torch.cat([sd[n].detach().reshape(-1).float().cpu() for n in self.param_names()]).numpy()

    def _handle(self, device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
        h = self._handles.get(idx)
        if h is None:
            h = _lib.CrnHandle(self.VERSION, self.config, self.dtype_name, idx, self.nlms)
            self._handles[idx] = h
        sd = self.state_dict(keep_vars=True)
        key = tuple((sd[n].data_ptr(), sd[n]._version) for n in self.param_names())
        if self._p_key.get(idx) != key:
            h.set_params(self.params_blob())
            self._p_key[idx] = key
        return h

    # ---- forward --------------------------------------------------------------
    def _check(self, *xs):
        if self.training:
            raise NotImplementedError('DCCRN (gfx950) is eval-mode inference only: call net.eval() '
                                      '(BatchNorm uses its running statistics)')
        if torch.is_grad_enabled() and any(x.requires_grad for x in xs if x is not None):
            raise NotImplementedError('DCCRN (gfx950) is inference-only: run under torch.no_grad()')
        dev = xs[0].device
        if dev.type != 'cuda':
            raise RuntimeError(f'DCCRN (gfx950) needs its inputs on a HIP device, got {dev}; there is no CPU path')
        for x in xs:
            if x is not None and (x.shape != xs[0].shape or x.device != dev):
                raise ValueError('mic, far, near and echo must share shape and device')
        return dev

    def spectra(self, x, lengths=None):
        """ConvSTFT (dccrn.py:45-52) on the GPU: [B, N] -> [B, 514, T]."""
        if x.dim() == 1:
            x = x[None]
        B, N = x.shape
        lengths = np.full(B, N, np.int64) if lengths is None else np.asarray(lengths, np.int64)
        T = int(lengths.max()) // HOP + 1
        h = self._handle(x.device)
        spec = torch.empty(B, T, 257, 2, device=x.device, dtype=torch.float32)
        x = x.contiguous().float()
        with torch.cuda.device(x.device):
            h.stft(x.data_ptr(), lengths, B, N, spec.data_ptr(), torch.cuda.current_stream(x.device).cuda_stream)
        return torch.cat([spec[..., 0], spec[..., 1]], dim=2).transpose(1, 2)

    def error_spectra(self, device):
        """NLMS networks: the FD-NLMS error spectrum E of the last forward on
        ``device`` (the spectrum the mask was applied to) -> [B, 514, T]."""
        if not self.nlms:
            raise RuntimeError('error_spectra needs a network built with nlms=...')
        dev = torch.device(device)
        h = self._handle(dev)
        B, T = self._last_shape[dev.index if dev.index is not None else torch.cuda.current_device()]
        spec = torch.empty(B, T, 257, 2, device=dev, dtype=torch.float32)
        with torch.cuda.device(dev):
            h.error_spec(spec.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        return torch.cat([spec[..., 0], spec[..., 1]], dim=2).transpose(1, 2)

    # ---- streaming (include/aec_crn.h aec_crn_stream_*) ------------------------
    def stream_open(self, B, device='cuda', graph=None):
        """Open B concurrent streams (state zeroed).  Then feed one 256-sample
        hop per stream per ``stream_step``; the output of step k is hop k-1 of
        the batch forward's out_wav (the first step's output is the trimmed
        warm-up region).  Feed N//256 + 1 hops per utterance, the last one
        zero-padded.  ``graph``: True replays each hop's launches from a
        hipGraph, False launches them directly, None keeps the library's
        choice (AEC_CRN_GRAPH, default direct); see ``stream_stats``."""
        self._check(torch.zeros(1, device=device))
        dev = torch.device(device)
        h = self._handle(dev)
        h.stream_open(B)
        if graph is not None:
            h.stream_set_graph(1 if graph else 0)
        self._stream = (h, dev, int(B))

    def stream_stats(self):
        """dict(graph_mode, graph_replays, direct_hops) since ``stream_open``."""
        return self._stream[0].stream_stats()

    def stream_reset(self, b=-1):
        h, dev, _ = self._stream
        with torch.cuda.device(dev):
            h.stream_reset(b, torch.cuda.current_stream(dev).cuda_stream)

    def stream_step(self, mic_hop, far_hop, out=None):
        """mic_hop / far_hop [B, 256] (row stride may exceed 256) -> out [B, 256]."""
        h, dev, B = self._stream                         # (parameters as of stream_open)
        if mic_hop.shape != (B, 256) or far_hop.shape != (B, 256):
            raise ValueError(f'hops must be [{B}, 256]')
        mic_hop = mic_hop.float()
        far_hop = far_hop.float()
        if mic_hop.stride(1) != 1 or far_hop.stride(1) != 1 or mic_hop.stride(0) != far_hop.stride(0):
            mic_hop, far_hop = mic_hop.contiguous(), far_hop.contiguous()
        out = torch.empty(B, 256, device=dev, dtype=torch.float32) if out is None else out
        with torch.cuda.device(dev):
            h.stream_step(mic_hop.data_ptr(), far_hop.data_ptr(), mic_hop.stride(0), out.data_ptr(), out.stride(0),
                          torch.cuda.current_stream(dev).cuda_stream)
        return out

    def forward_ragged(self, mic, far, lengths, want_spec=True, want_mask=False):
        """Rows zero-padded to a common width with true ``lengths``.  Returns
        (out_wav [B, 256*(max//256)] (row b valid to 256*(lengths[b]//256)),
        out_spec [B, 514, Tmax] or None, mask [B, 2, 256, Tmax] or None)."""
        dev = self._check(mic, far)
        mic = mic.contiguous().float()
        far = far.contiguous().float()
        B, N = mic.shape
        lengths = np.asarray(lengths, dtype=np.int64)
        if lengths.shape != (B,) or (lengths < 1).any() or (lengths > N).any():
            raise ValueError('lengths must be [B] with 1 <= length <= N')
        T = int(lengths.max()) // HOP + 1
        lout = HOP * (int(lengths.max()) // HOP)
        h = self._handle(dev)
        out = torch.zeros(B, lout, device=dev, dtype=torch.float32)
        spec = torch.empty(B, T, 257, 2, device=dev, dtype=torch.float32) if want_spec else None
        mask = torch.empty(B, T, 256, 2, device=dev, dtype=torch.float32) if want_mask else None
        with torch.cuda.device(dev):
            h.process(mic.data_ptr(), far.data_ptr(), lengths, B, N, out.data_ptr() if lout > 0 else None,
                      max(lout, 1), spec.data_ptr() if spec is not None else None,
                      mask.data_ptr() if mask is not None else None, torch.cuda.current_stream(dev).cuda_stream)
        self._last_shape[dev.index if dev.index is not None else torch.cuda.current_device()] = (B, T)
        out_spec = torch.cat([spec[..., 0], spec[..., 1]], dim=2).transpose(1, 2) if spec is not None else None
        mk = mask.permute(0, 3, 2, 1) if mask is not None else None
        return out, out_spec, mk


def _encoder_decoder(net, config, cbn):
    """Encoder / decoder construction in the reference's order
    (dccrn.py:463-509, dccrn2.py:49-111)."""
    ch = config['conv_channels']
    for i in range(len(ch) - 1):
        net.encoder.append(nn.Sequential(
            ComplexConv2d(ch[i], ch[i + 1], config['kernel_size'], config['stride'], config['padding'],
                          config['dilation'], config['groups']),
            ComplexBatchNorm(ch[i + 1]) if cbn else nn.BatchNorm2d(ch[i + 1]),
            nn.PReLU()))


def _check_fixed(config):
    if tuple(config['kernel_size']) != (5, 1) or tuple(config['stride']) != (2, 1) or \
            tuple(config['padding']) != (2, 0) or config.get('dilation', 1) != 1 or config.get('groups', 1) != 1:
        raise NotImplementedError('the gfx950 CRN implements kernel (5,1), stride (2,1), padding (2,0) '
                                  '(configs.net_conf)')
    if config['win_size'] != 512 or config['hop_size'] != 256:
        raise NotImplementedError('win 512 / hop 256 only (configs.net_conf)')
