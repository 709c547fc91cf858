"""``Little_net`` — drop-in for the reference's Stage-2 post-filter module.

Reference: ``Little_net`` in Stage2_lhm/scripts/network/ERB.py:203-334.

Same constructor ``Little_net(conf, erb_bands)``, same submodule / parameter /
buffer names (so the reference's ``state_dict`` loads with ``strict=True``,
scripts/test.py:124), same parameter init (orthogonal GRU weights, Kaiming
linears, ERB.py:226-250, in the same RNG order, so ``torch.manual_seed(s)``
gives the reference's weights), and the same
``forward(mic, ref, near, erb) -> (out_wav, loss)`` (ERB.py:252-334).

The forward runs entirely on the GPU through ``libaec_hip.so``; there is no
CPU fallback.  Per-stream semantics: every row of a [B, N] batch is processed
as the reference processes a batch of one (its normaliser uses the row's own
mean/std, ERB.py:254-256 at batch=1 — SURVEY.md §0.5).  ``loss`` is the sum of
the per-row losses, which equals the reference's value at B = 1.

Training (scripts/train1.py:191-218): in ``train()`` mode with gradients
enabled, ``forward`` follows the reference's training semantics on the padded
batch (one normaliser scalar per signal over the whole [B, N] tensor,
ERB.py:254-256; the batch-summed loss) through ``aec_train_forward``, and
``loss.backward()`` runs ``aec_train_backward`` (head + BPTT through the GRU
on the device) into the parameters' ``.grad`` — so the reference's loop
(``loss.backward(); optimizer.step()`` with ``torch.optim.Adam``) runs
unchanged.  ``aec_amd.train.Adam`` is the same optimizer as one HIP kernel.
The gradient flows through ``loss`` only (the reference never differentiates
``out_wav``); the inputs get no gradient.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import _lib

WIN, HOP = 512, 256


def _stft_bases():
    """Closed forms of the reference's fixed STFT buffers (attention_ccrn.py:8-25):
    forward rows [cos; -sin](2 pi k n / 512) * hann, inverse rows = irfft weights
    (c_k / 512, c_0 = c_256 = 1 else 2) * hann, i.e. pinv(forward).T * hann."""
    n = np.arange(WIN)
    k = np.arange(WIN // 2 + 1)[:, None]
    win = 0.5 - 0.5 * np.cos(2 * np.pi * n / WIN)
    ang = 2 * np.pi * k * n[None, :] / WIN
    fwd = np.concatenate([np.cos(ang), -np.sin(ang)], 0)
    ck = np.full((WIN // 2 + 1, 1), 2.0)
    ck[0] = ck[-1] = 1.0
    inv = np.concatenate([np.cos(ang) * ck, -np.sin(ang) * ck], 0) / WIN
    inv[WIN // 2 + 1] = 0.0          # imaginary DC row (pinv of an all-zero row)
    inv[-1] = 0.0                    # imaginary Nyquist row
    f32 = lambda a: torch.from_numpy((a * win).astype(np.float32))[:, None, :]
    return f32(fwd), f32(inv), torch.from_numpy(win.astype(np.float32))[None, :, None]


class _ConvSTFTBuffers(nn.Module):
    """Holds ``cpx_stft.weight`` [514,1,512] (attention_ccrn.py:36-38)."""

    def __init__(self, weight):
        super().__init__()
        self.register_buffer('weight', weight)


class _ConviSTFTBuffers(nn.Module):
    """Holds ``istft.weight`` / ``istft.window`` / ``istft.enframe`` (attention_ccrn.py:68-80)."""

    def __init__(self, weight, window):
        super().__init__()
        self.register_buffer('weight', weight)
        self.register_buffer('window', window)
        self.register_buffer('enframe', torch.eye(WIN)[:, None, :])


class _TrainStep(torch.autograd.Function):
    """forward: aec_train_forward; backward: aec_train_backward (include/aec_hip.h)."""

    @staticmethod
    def forward(ctx, net, mic, ref, near, erb, *params):
        ctx.set_materialize_grads(False)
        dev = mic.device
        h, idx = net._handle(dev, upload=False)
        net._sync_erb(h, idx, erb)
        stream = torch.cuda.current_stream(dev).cuda_stream
        blob = torch.cat([p.detach().reshape(-1).float() for p in params])
        B, N = mic.shape
        lout = HOP * (N // HOP)
        out = torch.empty(B, lout, device=dev, dtype=torch.float32)
        loss = torch.empty((), device=dev, dtype=torch.float32)
        with torch.cuda.device(dev):
            h.set_weights_device(blob.data_ptr(), blob.numel(), stream)
            h.train_forward(mic.data_ptr(), ref.data_ptr(), near.data_ptr(), N, B, N,
                            out.data_ptr() if lout > 0 else None, max(lout, 1), loss.data_ptr(), stream)
        net._w_key.pop(idx, None)        # the device blob no longer matches any host upload
        ctx.h, ctx.dev, ctx.gen = h, dev, h.train_generation()
        ctx.shapes = [p.shape for p in params]
        ctx.keep = (blob, mic, ref, near)   # the forward's buffers stay alive until the backward
        return out, loss

    @staticmethod
    def backward(ctx, g_out, g_loss):
        if g_out is not None:
            raise NotImplementedError('Little_net (gfx950) differentiates the loss only; the reference trains '
                                      'on loss (scripts/train1.py:207-212), not on out_wav')
        h, dev = ctx.h, ctx.dev
        if h.train_generation() != ctx.gen:
            raise RuntimeError('Little_net (gfx950): backward of an older forward (another forward ran on this '
                               'module and device in between); call backward before the next forward')
        grad = torch.empty(sum(int(np.prod(s)) for s in ctx.shapes), device=dev, dtype=torch.float32)
        gl = g_loss.detach().float().contiguous() if g_loss is not None else None
        stream = torch.cuda.current_stream(dev).cuda_stream
        with torch.cuda.device(dev):
            h.train_backward(gl.data_ptr() if gl is not None else None, grad.data_ptr(), stream)
        grads, o = [], 0
        for s in ctx.shapes:
            k = int(np.prod(s))
            grads.append(grad[o:o + k].view(s))
            o += k
        ctx.keep = None
        return (None, None, None, None, None, *grads)


class Little_net(nn.Module):
    def __init__(self, conf, erb_bands, nlms=None):
        super().__init__()
        self.config = conf
        self.win_len = conf['win_size']
        self.win_inc = conf['hop_size']
        if self.win_len != WIN or self.win_inc != HOP or erb_bands != 32:
            raise NotImplementedError('the gfx950 path implements win 512 / hop 256 / 32 ERB bands '
                                      '(speech_conf, erb_conf of the reference)')
        self.win_type = 'hann'
        # same module creation order as ERB.py:213-217 (RNG order matters for the init)
        self.gru1 = nn.GRU(2 * erb_bands, erb_bands, num_layers=1, batch_first=True, bias=True)
        self.linear1 = nn.Linear(2 * erb_bands, erb_bands, bias=True)
        self.linear2 = nn.Linear(erb_bands, erb_bands, bias=True)
        self.relu = nn.ReLU()
        self.sigmoid = nn.Sigmoid()
        fwd, inv, win = _stft_bases()
        self.cpx_stft = _ConvSTFTBuffers(fwd)
        self.istft = _ConviSTFTBuffers(inv, win)
        self.gru1.apply(self._orthogonal)
        self.linear1.apply(lambda m: self._kaiming(m, 'relu'))
        self.linear2.apply(lambda m: self._kaiming(m, 'sigmoid'))
        self.nlms = dict(nlms) if nlms else None
        self._handles = {}
        self._w_key = {}
        self._erb_key = {}

    # --- init, as ERB.py:231-250 -------------------------------------------
    @staticmethod
    def _kaiming(module, nonlinearity):
        if isinstance(module, nn.Linear):
            nn.init.kaiming_uniform_(module.weight, mode='fan_in', nonlinearity=nonlinearity)
            if module.bias is not None:
                nn.init.zeros_(module.bias)

    @staticmethod
    def _orthogonal(module):
        if isinstance(module, nn.GRU):
            for name, param in module.named_parameters():
                if 'weight' in name:
                    nn.init.orthogonal_(param.data)

    # --- device plumbing ------------------------------------------------------
    def _params(self):
        g = self.gru1
        return [g.weight_ih_l0, g.weight_hh_l0, g.bias_ih_l0, g.bias_hh_l0,
                self.linear1.weight, self.linear1.bias, self.linear2.weight, self.linear2.bias]

    def weights_blob(self):
        """The 12,544-float blob in state_dict order (include/aec_hip.h)."""
        return torch.cat([p.detach().reshape(-1).float().cpu() for p in self._params()]).numpy()

    def _handle(self, device, upload=True):
        idx = device.index if device.index is not None else torch.cuda.current_device()
        h = self._handles.get(idx)
        if h is None:
            nl = self.nlms or {}
            h = _lib.Handle(idx, nlms_taps=nl.get('taps', 0), nlms_mu=nl.get('mu', 0.5),
                            nlms_beta=nl.get('beta', 0.9), nlms_delta=nl.get('delta', 1e-4))
            self._handles[idx] = h
        if not upload:
            return h, idx
        wkey = tuple((p.data_ptr(), p._version) for p in self._params())
        if self._w_key.get(idx) != wkey:
            h.set_weights(self.weights_blob())
            self._w_key[idx] = wkey
        return h, idx

    def _sync_erb(self, h, idx, erb):
        key = (erb.data_ptr(), erb._version, str(erb.device), tuple(erb.shape))
        if self._erb_key.get(idx) != key:
            h.set_erb(erb.detach().float().cpu().numpy())
            self._erb_key[idx] = key

    def set_debug(self, on=True, device=None):
        device = torch.device(device or 'cuda')
        h, _ = self._handle(device)
        h.set_debug(on)

    # --- forward --------------------------------------------------------------
    def forward(self, mic, ref, near, erb):
        """(ERB.py:252-334) mic/ref/near [B, N] (or [N]) float32 on a HIP device."""
        if mic.dim() == 1:
            mic, ref, near = mic[None], ref[None], near[None] if near is not None else None
        if self.training and torch.is_grad_enabled() and any(p.requires_grad for p in self._params()):
            return self._train_forward(mic, ref, near, erb)
        B, N = mic.shape
        out, loss = self.forward_ragged(mic, ref, near, erb, [N] * B)
        return out, (loss.sum() if loss is not None else None)

    def _train_forward(self, mic, ref, near, erb):
        """Training semantics of the reference (scripts/train1.py:207-208): the
        padded [B, N] batch as ONE tensor (batch-global normaliser), the
        batch-summed loss; differentiable w.r.t. the 8 parameters."""
        if self.nlms:
            raise NotImplementedError('training covers the reference network (no FD-NLMS stage)')
        if near is None:
            raise ValueError('training needs near (the loss target)')
        dev = mic.device
        if dev.type != 'cuda':
            raise RuntimeError(f'Little_net (gfx950) needs its inputs on a HIP device, got {dev}; '
                               'there is no CPU path')
        if mic.requires_grad or ref.requires_grad or near.requires_grad:
            raise NotImplementedError('Little_net (gfx950) gives no gradient to its inputs')
        for t in (ref, near):
            if t.shape != mic.shape or t.device != dev:
                raise ValueError('mic, ref and near must share shape and device')
        if erb.shape != (257, 32):
            raise ValueError(f'erb must be [257, 32], got {tuple(erb.shape)}')
        params = self._params()
        if any(p.device != dev for p in params):
            raise RuntimeError('parameters and inputs must be on the same device (net.to(device))')
        mic, ref, near = (t.detach().contiguous().float() for t in (mic, ref, near))
        return _TrainStep.apply(self, mic, ref, near, erb, *params)

    def forward_ragged(self, mic, ref, near, erb, lengths, lookahead=None):
        """Batched call with per-row true lengths (rows zero-padded to a common
        width).  ``lengths`` is [B] (one length per row) or [B, 3] (mic, ref,
        near lengths of each row: every signal normalised over and padded
        beyond its own length, as test.py:139 feeds the reference; the three
        must share the frame count N//256 + 1).  Returns out
        [B, 256*(max(mic lengths)//256)] (row b valid up to 256*(n_mic//256),
        zero beyond) and per-row losses [B] (None when ``near`` is None).
        ``lookahead``: the token ``prepare_ragged`` returned for exactly these
        tensors and lengths; its queued normaliser pass is used instead of
        running one (a token that is not pending, or was prepared for other
        tensors / lengths, raises)."""
        if torch.is_grad_enabled() and (mic.requires_grad or any(p.requires_grad for p in self._params())
                                        and self.training):
            raise NotImplementedError('forward_ragged is the inference path (batch=1 semantics per row): call it '
                                      'under torch.no_grad() and net.eval(), as scripts/test.py:134,156 does; '
                                      'training goes through forward() in train() mode')
        dev = mic.device
        if dev.type != 'cuda':
            raise RuntimeError(f'Little_net (gfx950) needs its inputs on a HIP device, got {dev}; '
                               'there is no CPU path')
        tens = [mic, ref] + ([near] if near is not None else [])
        for t in tens:
            if t.shape != mic.shape or t.device != dev:
                raise ValueError('mic, ref and near must share shape and device')
        if erb.shape != (257, 32):
            raise ValueError(f'erb must be [257, 32], got {tuple(erb.shape)}')
        mic = mic.contiguous().float()
        ref = ref.contiguous().float()
        near = near.contiguous().float() if near is not None else None
        B, L = mic.shape
        lengths = np.asarray(lengths, dtype=np.int64)
        if lengths.shape not in ((B,), (B, 3)) or (lengths < 1).any() or (lengths > L).any():
            raise ValueError('lengths must be [B] or [B, 3] with 1 <= length <= N')
        nmic = lengths if lengths.ndim == 1 else lengths[:, 0]
        if lengths.ndim == 2:
            cols = [0, 1, 2] if near is not None else [0, 1]
            if (lengths[:, cols] // HOP != (nmic // HOP)[:, None]).any():
                # ERB.py:287-290 / 318-323 combine the signals frame by frame
                raise RuntimeError('mic, ref and near must have the same frame count N//256 + 1 '
                                   '(the reference raises on the shape mismatch)')
        h, idx = self._handle(dev)
        self._sync_erb(h, idx, erb)
        lout = HOP * (int(nmic.max()) // HOP)
        out = torch.zeros(B, lout, device=dev, dtype=torch.float32) if (nmic != nmic.max()).any() \
            else torch.empty(B, lout, device=dev, dtype=torch.float32)
        loss = torch.empty(B, device=dev, dtype=torch.float32) if near is not None else None
        stream = torch.cuda.current_stream(dev).cuda_stream
        if B > 0:
            with torch.cuda.device(dev):
                h.process(mic.data_ptr(), ref.data_ptr(), near.data_ptr() if near is not None else None,
                          lengths, B, L, out.data_ptr() if lout > 0 else None, max(lout, 1), loss.data_ptr() if loss is not None else None,
                          stream, token=lookahead or 0)
        return out, loss

    def prepare_ragged(self, mic, ref, near, lengths, producer=None):
        """Queue the normaliser pass (ERB.py:254-256) of a batch a later
        ``forward_ragged(..., lookahead=token)`` on this net takes, on the
        current stream (``aec_prepare_siglens``): a serving loop runs it on a
        side stream while the previous batch is still in flight.  Returns the
        token.  The tensors must be the very ones (contiguous float32, same
        data) passed to that ``forward_ragged``; a plain ``forward_ragged``
        never takes a look-ahead.  ``producer``: the stream that wrote the
        tensors (the pass waits for it; None = the caller has ordered them).
        The tensors are recorded on the current stream, so the caching
        allocator does not hand their memory out while the pass reads it.
        Outputs are bit-identical with and without the look-ahead."""
        dev = mic.device
        if dev.type != 'cuda':
            raise RuntimeError(f'Little_net (gfx950) needs its inputs on a HIP device, got {dev}')
        tens = [mic, ref] + ([near] if near is not None else [])
        for t in tens:
            if t.shape != mic.shape or t.device != dev or not t.is_contiguous() or t.dtype != torch.float32:
                raise ValueError('prepare_ragged needs contiguous float32 mic / ref / near of one shape and device')
        B, L = mic.shape
        lengths = np.asarray(lengths, dtype=np.int64)
        if lengths.shape not in ((B,), (B, 3)) or (lengths < 1).any() or (lengths > L).any():
            raise ValueError('lengths must be [B] or [B, 3] with 1 <= length <= N')
        h, _ = self._handle(dev)
        if B == 0:
            return 0
        cur = torch.cuda.current_stream(dev)
        if producer is not None:
            cur.wait_stream(producer)
        for t in tens:
            t.record_stream(cur)
        with torch.cuda.device(dev):
            return h.prepare(mic.data_ptr(), ref.data_ptr(), near.data_ptr() if near is not None else None,
                             lengths, B, L, cur.cuda_stream)

    # --- streaming (include/aec_hip.h aec_stream_*) ------------------------------
    def stream_open(self, B, erb, device=None):
        """Open B concurrent streams (state zeroed) on ``device``: afterwards
        ``stream_step`` advances every stream by one 256-sample hop."""
        if torch.is_grad_enabled() and self.training:
            raise NotImplementedError('streaming is inference-only: use net.eval() and torch.no_grad()')
        device = torch.device(device or 'cuda')
        if device.type != 'cuda':
            raise RuntimeError(f'Little_net (gfx950) streams live on a HIP device, got {device}')
        if erb.shape != (257, 32):
            raise ValueError(f'erb must be [257, 32], got {tuple(erb.shape)}')
        h, idx = self._handle(device)
        self._sync_erb(h, idx, erb)
        h.stream_open(B)
        self._stream = (h, torch.device('cuda', idx), int(B))

    def _stream_state(self):
        st = getattr(self, '_stream', None)
        if st is None:
            raise RuntimeError('call stream_open first')
        return st

    def stream_reset(self, b=-1):
        """Zero stream b's state (b = -1: every stream) for a new utterance."""
        h, device, _ = self._stream_state()
        h.stream_reset(b, torch.cuda.current_stream(device).cuda_stream)

    def stream_step(self, mic, ref):
        """mic, ref [B, 256] float32 (hop k of every stream, already normalised
        — see aec_stream_step) -> output hop k-1 [B, 256]."""
        h, device, B = self._stream_state()
        for t in (mic, ref):
            if t.device != device or t.dim() != 2 or t.shape[0] != B or t.shape[1] < HOP:
                raise ValueError(f'hops must be [{B}, >= 256] on {device}')
        mic = mic.float()
        ref = ref.float()
        if mic.stride(1) != 1 or ref.stride(1) != 1 or mic.stride(0) != ref.stride(0):
            mic, ref = mic.contiguous(), ref.contiguous()
        self._handle(device)            # weights may have changed
        out = torch.empty(B, HOP, device=device, dtype=torch.float32)
        with torch.cuda.device(device):
            h.stream_step(mic.data_ptr(), ref.data_ptr(), mic.stride(0), out.data_ptr(), HOP,
                          torch.cuda.current_stream(device).cuda_stream)
        return out

    def debug_intermediate(self, what, B, T, device=None):
        """Copy an intermediate of the last forward: 'mic_erb', 'ref_erb',
        'near_erb', 'gru_out', 'mask', 'est_erb' -> [B, T, 32]."""
        codes = dict(mic_erb=0, ref_erb=1, near_erb=2, gru_out=3, mask=4, est_erb=5)
        device = torch.device(device or 'cuda')
        h, _ = self._handle(device)
        dst = torch.empty(B, T, 32, device=device, dtype=torch.float32)
        h.debug_copy(codes[what], dst.data_ptr(), dst.numel(), torch.cuda.current_stream(device).cuda_stream)
        return dst
