"""CPU oracle for the Stage-2 AEC hot path — TEST INFRASTRUCTURE ONLY.

This module is the *checker*.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The product path
(``acoustic-echo-cancellation_amd/aec_amd``) never imports anything under
``oracle/`` and must fail loudly when its HIP library is missing.

It is a NumPy restatement (float64 by default) of the reference algorithm
``Little_net.forward`` in ``/root/reference/Stage2_lhm/scripts/network/ERB.py``
with its STFT modules from ``scripts/network/attention_ccrn.py``.  The
restatement replaces the reference's DFT-as-convolution with ``numpy.fft``
(rfft/irfft are algebraically identical to the reference's ``init_kernels``
bases) and its dense ERB matmuls with the same dense
product.

Parity pin: ``tests/test_oracle_golden.py`` checks every function here against
the golden vectors in ``tests/golden/`` that ``tests/golden/make_golden.py``
produced by importing and running the reference itself in the build container.

The FD-NLMS stage (``nlms_*``) has NO reference counterpart:
it is build-defined and its parity is *unpinned* against the reference; it is
pinned only by known-answer tests (mu=0 identity, convergence on a synthetic
echo path).
"""
from __future__ import annotations

import numpy as np

WIN = 512          # speech_conf['win_size']   (scripts/configs.py:6)
HOP = 256          # speech_conf['hop_size']   (scripts/configs.py:7)
NBIN = WIN // 2 + 1
NBAND = 32         # erb_conf['total_erb_bands'] (scripts/configs.py:24)


# --------------------------------------------------------------------------
# integer framing (bit-exact contract)
# --------------------------------------------------------------------------
def n_frames(n: int) -> int:
    """T for an N-sample input: F.pad(256,256) + conv1d(k=512, stride=256)
    (attention_ccrn.py:48-49) gives (N + 512 - 512)//256 + 1."""
    return n // HOP + 1


def out_len(n: int) -> int:
    """conv_transpose1d gives 256*(T+1) samples, trimmed by 256 at each end
    (attention_ccrn.py:92,99): 256*(T-1) = 256*(N//256)."""
    return HOP * (n_frames(n) - 1)


# --------------------------------------------------------------------------
# ERB filterbank — restates EquivalentRectangularBandwidth (ERB.py:10-71)
# --------------------------------------------------------------------------
_EARQ = 9.265
_MINBW = 24.7


def _f2e(f):
    return _EARQ * np.log(1.0 + np.asarray(f, dtype=np.float64) / (_MINBW * _EARQ))   # ERB.py:29-31


def _e2f(e):
    return (np.exp(np.asarray(e, dtype=np.float64) / _EARQ) - 1.0) * _MINBW * _EARQ   # ERB.py:33-35


def erb_filters(nfreqs=257, sample_rate=16000, bands=32, low_freq=0, max_freq=8000):
    """cos_filts [nfreqs, bands] float64 (ERB.py:10-27,37-58,71).  Only the
    cosine lobes are returned; the LP/HP edge filters are discarded (:60-71)."""
    if low_freq is None:
        low_freq = 20
    if max_freq is None:
        max_freq = sample_rate // 2
    freqs = np.linspace(0, max_freq, nfreqs)
    cut = _e2f(np.linspace(_f2e(low_freq), _f2e(max_freq), bands + 2))
    out = np.zeros((nfreqs, bands))
    for i in range(bands):
        lo, hi = cut[i], cut[i + 2]
        a = int(np.min(np.where(freqs > lo)))
        b = int(np.max(np.where(freqs < hi)))
        mid = (_f2e(lo) + _f2e(hi)) / 2
        span = _f2e(hi) - _f2e(lo)
        out[a:b + 1, i] = np.cos((_f2e(freqs[a:b + 1]) - mid) / span * np.pi)
    return out


# --------------------------------------------------------------------------
# STFT pieces — restate ConvSTFT / ConviSTFT (attention_ccrn.py:8-101)
# --------------------------------------------------------------------------
def hann(dtype=np.float64):
    """scipy.signal.get_window('hann', 512, fftbins=True) (attention_ccrn.py:12):
    the periodic Hann window 0.5 - 0.5 cos(2 pi n / 512)."""
    n = np.arange(WIN)
    return (0.5 - 0.5 * np.cos(2.0 * np.pi * n / WIN)).astype(dtype)


def normalise(x):
    """x - mean(x)/std(x) over the WHOLE array, unbiased std (ERB.py:254-256).
    Called per stream (batch=1 semantics)."""
    x = np.asarray(x, dtype=np.float64)
    return x - x.mean() / x.std(ddof=1)


def stft(x):
    """[N] -> complex [T, 257]: zero-pad 256 both sides, frame t = padded
    [256t, 256t+512), periodic-Hann window, rfft-512 (attention_ccrn.py:45-52)."""
    x = np.asarray(x, dtype=np.float64)
    n = x.shape[-1]
    T = n_frames(n)
    xp = np.pad(x, (WIN - HOP, WIN - HOP))
    idx = np.arange(T)[:, None] * HOP + np.arange(WIN)[None, :]
    return np.fft.rfft(xp[idx] * hann(), axis=-1)


def magnitude(spec):
    """sqrt(re^2 + im^2 + 1e-9) (ERB.py:277-279)."""
    return np.sqrt(spec.real ** 2 + spec.imag ** 2 + 1e-9)


def istft(spec, n):
    """complex [T,257] -> [256*(T-1)] : windowed irfft frames, overlap-add,
    divide by (sum of shifted window^2 + 1e-8), trim 256 both ends
    (attention_ccrn.py:82-101).  DC/Nyquist imaginary parts are ignored
    exactly as the pinv basis ignores them (its columns for those rows are 0)."""
    T = spec.shape[0]
    w = hann()
    frames = np.fft.irfft(spec, n=WIN, axis=-1) * w
    L = HOP * (T + 1)
    ola = np.zeros(L)
    coff = np.zeros(L)
    w32 = hann(np.float32).astype(np.float64)   # coff uses the f32 window buffer
    for t in range(T):
        ola[t * HOP:t * HOP + WIN] += frames[t]
        coff[t * HOP:t * HOP + WIN] += w32 ** 2
    y = ola / (coff + 1e-8)
    return y[WIN - HOP:L - (WIN - HOP)]


# --------------------------------------------------------------------------
# recurrent + head — nn.GRU(64,32) and the 2 linears (ERB.py:213-217,293-301)
# --------------------------------------------------------------------------
def _sig(v):
    return 1.0 / (1.0 + np.exp(-v))


def gru(x, w_ih, w_hh, b_ih, b_hh):
    """PyTorch GRU, gate order (r, z, n), h0 = 0.  x [T,64] -> h [T,32]."""
    x = np.asarray(x, np.float64)
    w_ih, w_hh = np.asarray(w_ih, np.float64), np.asarray(w_hh, np.float64)
    b_ih, b_hh = np.asarray(b_ih, np.float64), np.asarray(b_hh, np.float64)
    H = w_hh.shape[1]
    gi = x @ w_ih.T + b_ih
    h = np.zeros(H)
    out = np.zeros((x.shape[0], H))
    for t in range(x.shape[0]):
        gh = w_hh @ h + b_hh
        r = _sig(gi[t, :H] + gh[:H])
        z = _sig(gi[t, H:2 * H] + gh[H:2 * H])
        nn_ = np.tanh(gi[t, 2 * H:] + r * gh[2 * H:])
        h = (1.0 - z) * nn_ + z * h
        out[t] = h
    return out


def little_net_forward(mic, ref, near, erb, w, return_intermediates=False):
    """Restatement of Little_net.forward (ERB.py:252-334) for ONE utterance.

    mic/ref/near: [N] arrays; erb: [257,32]; w: dict with the reference
    state_dict names (gru1.weight_ih_l0 ... linear2.bias).
    Returns (out [256*(N//256)], loss) and optionally the intermediates."""
    n = len(mic)
    erb = np.asarray(erb, np.float64)
    S_mic = stft(normalise(mic))
    S_ref = stft(normalise(ref))
    S_near = stft(normalise(near))
    mic_erb = magnitude(S_mic) @ erb                                     # :282
    ref_erb = magnitude(S_ref) @ erb                                     # :283
    near_erb = magnitude(S_near) @ erb                                   # :284
    x = np.concatenate([mic_erb, np.abs(mic_erb - ref_erb)], axis=1)     # :287-290
    h = gru(x, w['gru1.weight_ih_l0'], w['gru1.weight_hh_l0'],
            w['gru1.bias_ih_l0'], w['gru1.bias_hh_l0'])                  # :293
    hc = np.concatenate([h, mic_erb], axis=1)                            # :295
    o = np.maximum(hc @ np.asarray(w['linear1.weight'], np.float64).T
                   + np.asarray(w['linear1.bias'], np.float64), 0.0)     # :298
    mask = _sig(o @ np.asarray(w['linear2.weight'], np.float64).T
                + np.asarray(w['linear2.bias'], np.float64))             # :301
    est_erb = mask * mic_erb                                             # :304
    gain = est_erb @ erb.T                                               # :306-307
    out = istft(gain * S_mic, n) + 1e-9                                  # :309-316
    T = S_mic.shape[0]
    loss = np.sum((near_erb ** 0.5 - est_erb ** 0.5) ** 2) / (T * erb.shape[1])   # :318-323
    if not return_intermediates:
        return out, loss
    return out, loss, dict(mic_erb=mic_erb, ref_erb=ref_erb, near_erb=near_erb,
                           gru_in=x, gru_out=h, mask=mask, est_erb=est_erb)


# --------------------------------------------------------------------------
# FD-NLMS — build-defined (no reference counterpart; parity UNPINNED)
# --------------------------------------------------------------------------
def nlms(S_mic, S_ref, taps=4, mu=0.3, beta=0.5, delta=1e-4):
    """Per-bin complex NLMS over frames (float64).

    For every bin k and frame t (tap l uses the far-end spectrum l frames back,
    zero before the first frame):
        Yhat = sum_l W[l] * R[t-l]
        E[t] = D[t] - Yhat                                   (a-priori error = output)
        P    = beta * P + (1 - beta) * sum_l |R[t-l]|^2      (P starts at 0)
        W[l] += mu * E[t] * conj(R[t-l]) / (P + delta)
    Returns E [T,257] complex."""
    S_mic = np.asarray(S_mic, np.complex128)
    S_ref = np.asarray(S_ref, np.complex128)
    T, K = S_mic.shape
    W = np.zeros((taps, K), np.complex128)
    P = np.zeros(K)
    hist = np.zeros((taps, K), np.complex128)       # hist[l] = R[t-l]
    E = np.zeros_like(S_mic)
    for t in range(T):
        hist = np.roll(hist, 1, axis=0)
        hist[0] = S_ref[t]
        yhat = np.sum(W * hist, axis=0)
        e = S_mic[t] - yhat
        P = beta * P + (1.0 - beta) * np.sum(np.abs(hist) ** 2, axis=0)
        W = W + mu * e[None, :] * np.conj(hist) / (P + delta)[None, :]
        E[t] = e
    return E


def aec_forward(mic, ref, near, erb, w, nlms_cfg=None):
    """Full build pipeline for one utterance: STFT -> [FD-NLMS] -> ERB-GRU
    post-filter -> iSTFT.  With nlms_cfg=None this IS little_net_forward."""
    if nlms_cfg is None:
        return little_net_forward(mic, ref, near, erb, w)
    n = len(mic)
    erb = np.asarray(erb, np.float64)
    S_mic = stft(normalise(mic))
    S_ref = stft(normalise(ref))
    S_near = stft(normalise(near))
    E = nlms(S_mic, S_ref, **nlms_cfg)
    mic_erb = magnitude(E) @ erb
    ref_erb = magnitude(S_ref) @ erb
    near_erb = magnitude(S_near) @ erb
    x = np.concatenate([mic_erb, np.abs(mic_erb - ref_erb)], axis=1)
    h = gru(x, w['gru1.weight_ih_l0'], w['gru1.weight_hh_l0'],
            w['gru1.bias_ih_l0'], w['gru1.bias_hh_l0'])
    hc = np.concatenate([h, mic_erb], axis=1)
    o = np.maximum(hc @ np.asarray(w['linear1.weight'], np.float64).T
                   + np.asarray(w['linear1.bias'], np.float64), 0.0)
    mask = _sig(o @ np.asarray(w['linear2.weight'], np.float64).T
                + np.asarray(w['linear2.bias'], np.float64))
    est_erb = mask * mic_erb
    out = istft((est_erb @ erb.T) * E, n) + 1e-9
    T = E.shape[0]
    loss = np.sum((near_erb ** 0.5 - est_erb ** 0.5) ** 2) / (T * erb.shape[1])
    return out, loss


def erle_db(mic, out, skip=8000):
    """ERLE = 10 log10(sum mic^2 / sum out^2) over n < len(out), skipping the
    first `skip` samples."""
    L = len(out)
    m = np.asarray(mic[:L], np.float64)[skip:]
    o = np.asarray(out, np.float64)[skip:]
    return 10.0 * np.log10(np.sum(m * m) / max(np.sum(o * o), 1e-30))
