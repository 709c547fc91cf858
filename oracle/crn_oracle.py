"""CPU oracle for the DCCRN (CRN) post-filter — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module; the product path never does.

A float64 NumPy restatement of the reference's two complex CRNs, eval mode
(SURVEY.md §8 a14):

* ``dccrn``  — ``Stage2_lhm/scripts/network/dccrn.py:453-594``: 6 x
  (ComplexConv2d + BatchNorm2d + PReLU) encoder, one real LSTM over the
  flattened [C, F] map, 6 x (ComplexConvTranspose2d + BatchNorm2d + PReLU,
  last: + BatchNorm2d(2) + Tanh) decoder with complex_cat skips, mask 'C',
  plus the training loss (cIRM MSE + masked-echo energy, :556-581);
* ``dccrn2`` — ``Stage2_lhm/scripts/network/dccrn2.py:10-218``: the same
  encoder/decoder with ComplexBatchNorm (``use_cbn``) or BatchNorm2d, 2 x
  NavieComplexLSTM (``dccrn.py:423-450``), last decoder layer bare, masks
  'E' / 'C' / 'R' (dccrn2.py:194-210).

Layout follows the reference: feature maps are [C, F, T] per utterance
(batch = 1; nothing in either model couples utterances in eval mode).
Parity pin: ``tests/test_crn_oracle.py`` checks this module against
``tests/golden/crn_*.npz``, which ``tests/golden/make_crn_golden.py``
produced by importing and running the reference modules themselves with the
weights of ``make_weights`` loaded through ``load_state_dict``.
"""
from __future__ import annotations

import numpy as np

from aec_oracle import HOP, WIN, istft, n_frames, stft   # noqa: F401  (shared STFT restatement)

# scripts/configs.py:29-46 (net_conf)
NET_CONF = {
    'win_size': 512, 'hop_size': 256, 'samplerates': 16000, 'win_type': 'hann',
    'hidden_dim': 4, 'rnn_layers': 2, 'rnn_units': 128, 'use_clstm': True, 'use_cbn': True,
    'masking_mode': 'E', 'conv_channels': [4, 16, 32, 64, 128, 256, 512],
    'kernel_size': (5, 1), 'stride': (2, 1), 'padding': (2, 0), 'dilation': 1, 'groups': 1,
}


# --------------------------------------------------------------------------
# parameter naming / seeded fixture weights
# --------------------------------------------------------------------------
def param_shapes(conf, version):
    """Ordered (name, shape) of the reference state_dict entries the forward
    reads (STFT buffers excluded: closed form, see aec_oracle)."""
    ch = list(conf['conv_channels'])
    L = len(ch) - 1
    out = []
    cbn = version == 2 and conf['use_cbn']

    def norm(prefix, c):
        if cbn:    # ComplexBatchNorm (dccrn.py:210-253): num_features = c // 2
            for n in ('Wrr', 'Wri', 'Wii', 'Br', 'Bi', 'RMr', 'RMi', 'RVrr', 'RVri', 'RVii'):
                out.append((f'{prefix}.{n}', (c // 2,)))
        else:      # nn.BatchNorm2d(c)
            for n in ('weight', 'bias', 'running_mean', 'running_var'):
                out.append((f'{prefix}.{n}', (c,)))

    for i in range(L):          # encoder (dccrn.py:463-476, dccrn2.py:49-62)
        ci, co = ch[i] // 2, ch[i + 1] // 2
        for part in ('real_conv', 'imag_conv'):
            out.append((f'encoder.{i}.0.{part}.weight', (co, ci, 5, 1)))
            out.append((f'encoder.{i}.0.{part}.bias', (co,)))
        norm(f'encoder.{i}.1', ch[i + 1])
        out.append((f'encoder.{i}.2.weight', (1,)))
    for d, c in enumerate(range(L, 0, -1)):   # decoder (dccrn.py:479-509, dccrn2.py:83-111)
        ci = ch[c]                      # (2*ch[c]) // 2
        co = (ch[c - 1] if c != 1 else 2) // 2
        for part in ('real_conv', 'imag_conv'):
            out.append((f'decoder.{d}.0.{part}.weight', (ci, co, 5, 1)))
            out.append((f'decoder.{d}.0.{part}.bias', (co,)))
        if c != 1:
            norm(f'decoder.{d}.1', ch[c - 1])
            out.append((f'decoder.{d}.2.weight', (1,)))
        elif version == 1:
            norm(f'decoder.{d}.1', 2)   # BatchNorm2d(2) + Tanh (dccrn.py:494-506)
    if version == 1:            # nn.LSTM(C*4, C*4) (dccrn.py:514)
        H = ch[-1] * 4
        out += [('lstm.weight_ih_l0', (4 * H, H)), ('lstm.weight_hh_l0', (4 * H, H)),
                ('lstm.bias_ih_l0', (4 * H,)), ('lstm.bias_hh_l0', (4 * H,))]
    else:                       # rnn_layers x NavieComplexLSTM(hidden_dim*C) (dccrn2.py:67-78)
        H = conf['hidden_dim'] * ch[-1] // 2
        for l in range(conf['rnn_layers']):
            for part in ('real_lstm', 'imag_lstm'):
                p = f'enhance.{l}.{part}'
                out += [(f'{p}.weight_ih_l0', (4 * H, H)), (f'{p}.weight_hh_l0', (4 * H, H)),
                        (f'{p}.bias_ih_l0', (4 * H,)), (f'{p}.bias_hh_l0', (4 * H,))]
    return out


def make_weights(conf, version, seed):
    """Deterministic fixture weights (float32) with the reference's init
    scales (conv N(0, 0.05), dccrn.py:135-138 / :178-181; LSTM U(+-1/sqrt(H)))
    and NON-trivial eval statistics for every (Complex)BatchNorm so the
    folding is exercised (positive-definite 2x2 running covariances)."""
    rng = np.random.default_rng(seed)
    w = {}
    for name, shape in param_shapes(conf, version):
        leaf = name.rsplit('.', 1)[1]
        if 'lstm' in name:
            H = shape[-1] if len(shape) == 2 else shape[0] // 4
            v = rng.uniform(-1, 1, shape) / np.sqrt(H)
        elif name.endswith('conv.weight'):
            v = rng.standard_normal(shape) * 0.05
        elif name.endswith('conv.bias'):
            v = rng.standard_normal(shape) * 0.02
        elif leaf in ('Wrr', 'Wii'):
            v = rng.uniform(0.8, 1.2, shape)
        elif leaf == 'Wri':
            v = rng.uniform(-0.3, 0.3, shape)
        elif leaf in ('Br', 'Bi', 'RMr', 'RMi', 'bias', 'running_mean'):
            v = rng.standard_normal(shape) * 0.05
        elif leaf in ('RVrr', 'RVii', 'running_var'):
            v = rng.uniform(0.5, 1.5, shape)
        elif leaf == 'RVri':
            v = rng.uniform(-0.3, 0.3, shape)
        elif leaf == 'weight' and shape == (1,):      # PReLU
            v = rng.uniform(0.1, 0.3, shape)
        elif leaf == 'weight':                        # BatchNorm2d affine
            v = rng.uniform(0.8, 1.2, shape)
        else:
            raise KeyError(name)
        w[name] = v.astype(np.float32)
    return w


# --------------------------------------------------------------------------
# layers ([C, F, T] maps, float64)
# --------------------------------------------------------------------------
def conv_f(x, W, b):
    """nn.Conv2d(k=(5,1), s=(2,1), p=(2,0)) over the frequency axis:
    x [Ci, F, T], W [Co, Ci, 5, 1] -> [Co, F//2 (ceil), T]."""
    Ci, F, T = x.shape
    Fo = (F + 4 - 5) // 2 + 1
    xp = np.pad(x, ((0, 0), (2, 2), (0, 0)))
    cols = np.stack([xp[:, k:k + 2 * Fo:2, :] for k in range(5)], axis=1)   # [Ci, 5, Fo, T]
    return np.einsum('oik,ikft->oft', W[..., 0].astype(np.float64), cols) + b[:, None, None]


def convT_f(x, W, b):
    """nn.ConvTranspose2d(k=(5,1), s=(2,1), p=(2,0), output_padding=(1,0)):
    x [Ci, F, T], W [Ci, Co, 5, 1] -> [Co, 2F, T]."""
    Ci, F, T = x.shape
    Co = W.shape[1]
    full = np.zeros((Co, 2 * F + 4, T))
    for k in range(5):
        full[:, k:k + 2 * F:2, :] += np.einsum('io,ift->oft', W[:, :, k, 0].astype(np.float64), x)
    return full[:, 2:2 + 2 * F, :] + b[:, None, None]


def complex_apply(f, x, w, prefix):
    """ComplexConv2d / ComplexConvTranspose2d forward (dccrn.py:140-153,
    :194-207): real = r(x_r) - i(x_i), imag = i(x_r) + r(x_i), each conv with
    its own bias."""
    C = x.shape[0] // 2
    xr, xi = x[:C], x[C:]
    R = lambda z: f(z, w[f'{prefix}.real_conv.weight'], w[f'{prefix}.real_conv.bias'].astype(np.float64))
    I = lambda z: f(z, w[f'{prefix}.imag_conv.weight'], w[f'{prefix}.imag_conv.bias'].astype(np.float64))
    return np.concatenate([R(xr) - I(xi), I(xr) + R(xi)], axis=0)


def batchnorm(x, w, prefix, eps=1e-5):
    """nn.BatchNorm2d eval: (x - running_mean)/sqrt(running_var + eps)*weight + bias."""
    g = lambda n: w[f'{prefix}.{n}'].astype(np.float64)[:, None, None]
    return (x - g('running_mean')) / np.sqrt(g('running_var') + eps) * g('weight') + g('bias')


def complex_batchnorm(x, w, prefix, eps=1e-5):
    """ComplexBatchNorm eval (dccrn.py:255-383): whitening by the running
    2x2 covariance, then the affine 2x2 W and bias."""
    C = x.shape[0] // 2
    xr, xi = x[:C], x[C:]
    g = lambda n: w[f'{prefix}.{n}'].astype(np.float64)[:, None, None]
    xr, xi = xr - g('RMr'), xi - g('RMi')
    Vrr, Vri, Vii = g('RVrr') + eps, g('RVri'), g('RVii') + eps
    tau = Vrr + Vii
    s = np.sqrt(Vrr * Vii - Vri * Vri)
    t = np.sqrt(tau + 2 * s)
    rst = 1.0 / (s * t)
    Urr, Uii, Uri = (s + Vii) * rst, (s + Vrr) * rst, -Vri * rst
    Wrr, Wri, Wii = g('Wrr'), g('Wri'), g('Wii')
    Zrr = Wrr * Urr + Wri * Uri
    Zri = Wrr * Uri + Wri * Uii
    Zir = Wri * Urr + Wii * Uri
    Zii = Wri * Uri + Wii * Uii
    yr = Zrr * xr + Zri * xi + g('Br')
    yi = Zir * xr + Zii * xi + g('Bi')
    return np.concatenate([yr, yi], axis=0)


def prelu(x, a):
    return np.where(x >= 0, x, float(a[0]) * x)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm(x, w, prefix):
    """nn.LSTM, one layer, h0 = c0 = 0, gate order (i, f, g, o):
    x [T, I] -> h [T, H]."""
    Wih = w[f'{prefix}.weight_ih_l0'].astype(np.float64)
    Whh = w[f'{prefix}.weight_hh_l0'].astype(np.float64)
    b = w[f'{prefix}.bias_ih_l0'].astype(np.float64) + w[f'{prefix}.bias_hh_l0'].astype(np.float64)
    H = Whh.shape[1]
    gx = x @ Wih.T + b
    h = np.zeros(H)
    c = np.zeros(H)
    out = np.empty((x.shape[0], H))
    for t in range(x.shape[0]):
        gt = gx[t] + Whh @ h
        i, f, gg, o = sigmoid(gt[:H]), sigmoid(gt[H:2 * H]), np.tanh(gt[2 * H:3 * H]), sigmoid(gt[3 * H:])
        c = f * c + i * gg
        h = o * np.tanh(c)
        out[t] = h
    return out


def complex_cat(a, b):
    """complex_cat([a, b], 1) (dccrn.py:386-395): [a_r, b_r, a_i, b_i]."""
    ca, cb = a.shape[0] // 2, b.shape[0] // 2
    return np.concatenate([a[:ca], b[:cb], a[ca:], b[cb:]], axis=0)


# --------------------------------------------------------------------------
# forward passes
# --------------------------------------------------------------------------
def _encode(w, conf, version, cspecs):
    cbn = version == 2 and conf['use_cbn']
    out = cspecs
    skips = []
    for i in range(len(conf['conv_channels']) - 1):
        out = complex_apply(conv_f, out, w, f'encoder.{i}.0')
        out = complex_batchnorm(out, w, f'encoder.{i}.1') if cbn else batchnorm(out, w, f'encoder.{i}.1')
        out = prelu(out, w[f'encoder.{i}.2.weight'])
        skips.append(out)
    return out, skips


def _decode(w, conf, version, out, skips):
    cbn = version == 2 and conf['use_cbn']
    L = len(conf['conv_channels']) - 1
    for d in range(L):
        out = complex_cat(out, skips[-1 - d])
        out = complex_apply(convT_f, out, w, f'decoder.{d}.0')
        if d != L - 1:
            out = complex_batchnorm(out, w, f'decoder.{d}.1') if cbn else batchnorm(out, w, f'decoder.{d}.1')
            out = prelu(out, w[f'decoder.{d}.2.weight'])
        elif version == 1:
            out = np.tanh(batchnorm(out, w, f'decoder.{d}.1'))
    return out


def _specs(x):
    s = stft(x).T            # [257, T]
    return s.real, s.imag


def apply_mask(mode, mr, mi, xr, xi):
    """mask_real/mask_imag [256, T] (DC bin excluded) -> est spectrum [257, T]
    (dccrn.py:575,585-590; dccrn2.py:189-210)."""
    mr = np.pad(mr, ((1, 0), (0, 0)))
    mi = np.pad(mi, ((1, 0), (0, 0)))
    if mode == 'E':
        mags = np.sqrt(xr ** 2 + xi ** 2 + 1e-8)
        phase = np.arctan2(xi, xr)
        mm = np.sqrt(mr ** 2 + mi ** 2)
        mphase = np.arctan2(mi / (mm + 1e-8), mr / (mm + 1e-8))
        em = np.tanh(mm) * mags
        ph = phase + mphase
        return em * np.cos(ph), em * np.sin(ph)
    if mode == 'C':
        return xr * mr - xi * mi, xr * mi + xi * mr
    if mode == 'R':
        return xr * mr, xi * mi
    raise ValueError(mode)


def forward(w, conf, version, mic, far, near=None, echo=None, capture=None, nlms=None):
    """One utterance through DCCRN (version 1: dccrn.py, 2: dccrn2.py), eval.

    nlms: None (the reference network) or dict(taps, mu, beta, delta): the
    build-defined FD-NLMS front end (include/aec_crn.h) — the mic spectrum is
    replaced everywhere below (encoder input, masking, the v1 loss's cRM
    reference) by the a-priori error of aec_oracle.nlms driven by the far
    spectrum.

    Returns dict(out_wav [256*(N//256)], out_spec [514, T], near_spec
    [514, T] or None, mask [2, 256, T], loss (version 1 with near and echo),
    err_spec [514, T] with nlms).
    """
    n = len(mic)
    mr_, mi_ = _specs(mic)
    fr_, fi_ = _specs(far)
    err_spec = None
    if nlms:
        from aec_oracle import nlms as _nlms
        E = _nlms((mr_ + 1j * mi_).T, (fr_ + 1j * fi_).T, taps=nlms.get('taps', 4), mu=nlms.get('mu', 0.3),
                  beta=nlms.get('beta', 0.5), delta=nlms.get('delta', 1e-4)).T
        mr_, mi_ = E.real.copy(), E.imag.copy()
        err_spec = np.concatenate([mr_, mi_], axis=0)
    cs = np.stack([mr_, fr_, mi_, fi_], axis=0)[:, 1:, :]   # [4, 256, T] (dccrn.py:560-561)
    enc, skips = _encode(w, conf, version, cs)
    C, D, T = enc.shape
    if version == 1:
        x = enc.transpose(2, 0, 1).reshape(T, C * D)         # [T, C*D] (dccrn.py:569-571)
        y = lstm(x, w, 'lstm')
        rnn = y.reshape(T, C, D).transpose(1, 2, 0)
    else:
        xr = enc[:C // 2].transpose(2, 0, 1).reshape(T, -1)  # dccrn2.py:147-151
        xi = enc[C // 2:].transpose(2, 0, 1).reshape(T, -1)
        for l in range(conf['rnn_layers']):                  # NavieComplexLSTM (dccrn.py:438-446)
            p = f'enhance.{l}'
            rr, ri = lstm(xr, w, f'{p}.real_lstm'), lstm(xr, w, f'{p}.imag_lstm')
            ir, ii = lstm(xi, w, f'{p}.real_lstm'), lstm(xi, w, f'{p}.imag_lstm')
            xr, xi = rr - ii, ir + ri
        rnn = np.concatenate([xr.reshape(T, C // 2, D), xi.reshape(T, C // 2, D)], axis=1).transpose(1, 2, 0)
    if capture is not None:
        capture['enc'] = skips
        capture['rnn'] = rnn
    dec = _decode(w, conf, version, rnn, skips)              # [2, 256, T]
    mode = 'C' if version == 1 else conf['masking_mode']
    er, ei = apply_mask(mode, dec[0], dec[1], mr_, mi_)
    out_spec = np.concatenate([er, ei], axis=0)
    out_wav = istft((er + 1j * ei).T, n)
    res = dict(out_wav=out_wav, out_spec=out_spec, mask=dec, near_spec=None, loss=None, err_spec=err_spec)
    if near is not None:
        nr, ni = _specs(near)
        res['near_spec'] = np.concatenate([nr, ni], axis=0)
        if version == 1 and echo is not None:              # dccrn.py:556-581
            er_, ei_ = _specs(echo)
            den = mr_ ** 2 + mi_ ** 2 + 1e-9
            cr = (mr_ * nr + mi_ * ni) / den
            ci = (mr_ * ni - mi_ * nr) / den
            mkr, mki = np.pad(dec[0], ((1, 0), (0, 0))), np.pad(dec[1], ((1, 0), (0, 0)))
            loss_mask = np.mean((mkr - cr) ** 2) + np.mean((mki - ci) ** 2)
            xr2 = er_ * mkr - ei_ * mki
            xi2 = er_ * mki + ei_ * mkr
            loss_echo = np.mean(xr2 ** 2) + np.mean(xi2 ** 2)
            res['loss'] = 0.3 * loss_mask + 0.7 * loss_echo
    return res
