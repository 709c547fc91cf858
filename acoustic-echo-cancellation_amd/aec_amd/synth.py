"""Synthetic 16 kHz far-end / near-end scenes (SURVEY.md §8(d) "Synthetic inputs").

The reference ships no audio, so benches and tests use seeded
scenes built here:

* far-end ``ref``: AR(1)-coloured Gaussian (a = 0.9) under a 4 Hz
  syllable-like envelope, scaled to 0.1 RMS;
* ``echo`` = ref * RIR, RIR = 1,024 taps, exponential decay (T60 ~ 0.25 s),
  random sign, 8 ms pure delay, scaled to -6 dB relative to ref;
* ``near``: zeros (far-end single talk, ERLE runs) or independent coloured
  bursts at -3 dB (double talk);
* ``mic`` = echo + near + white noise at -50 dB.

Everything is float32 and fully determined by ``seed`` (numpy PCG64).
"""
from __future__ import annotations

import numpy as np

SR = 16000


def _ar1(rng, n, a=0.9):
    w = rng.standard_normal(n)
    # y[t] = a y[t-1] + w[t] via a short IIR run in float64
    from scipy.signal import lfilter
    return lfilter([1.0], [1.0, -a], w)


def _envelope(rng, n, rate_hz=4.0):
    t = np.arange(n) / SR
    ph = rng.uniform(0, 2 * np.pi)
    return 0.55 + 0.45 * np.sin(2 * np.pi * rate_hz * t + ph)


def rir(rng, taps=1024, t60=0.25, delay_ms=8.0):
    d = int(round(delay_ms * 1e-3 * SR))
    n = np.arange(taps - d)
    decay = np.exp(-6.9078 * n / (t60 * SR))          # 60 dB over t60
    h = np.zeros(taps)
    h[d:] = decay * rng.choice([-1.0, 1.0], size=taps - d) * rng.uniform(0.5, 1.0, taps - d)
    return h / np.sqrt(np.sum(h * h))


def _rms(x):
    return float(np.sqrt(np.mean(np.square(x)) + 1e-30))


def scene(n, seed, double_talk=True, return_echo=False):
    """Return float32 (mic, ref, near[, echo]) of length n."""
    from scipy.signal import fftconvolve
    rng = np.random.default_rng(seed)
    ref = _ar1(rng, n) * _envelope(rng, n)
    ref *= 0.1 / _rms(ref)
    h = rir(rng)
    echo = fftconvolve(ref, h)[:n]
    echo *= (_rms(ref) * 10 ** (-6 / 20)) / _rms(echo)
    if double_talk:
        near = _ar1(rng, n, a=0.7) * _envelope(rng, n, rate_hz=2.5)
        gate = (np.sin(2 * np.pi * 0.4 * np.arange(n) / SR + rng.uniform(0, 6.28)) > 0.2)
        near *= gate
        near *= (_rms(ref) * 10 ** (-3 / 20)) / max(_rms(near), 1e-12)
    else:
        near = np.zeros(n)
    noise = rng.standard_normal(n) * _rms(ref) * 10 ** (-50 / 20)
    mic = echo + near + noise
    out = (mic.astype(np.float32), ref.astype(np.float32), near.astype(np.float32))
    if return_echo:
        out = out + (echo.astype(np.float32),)
    return out


def batch(B, n, seed0=0, double_talk=True):
    """[B, n] float32 arrays (mic, ref, near) with per-stream seeds seed0+b."""
    mic = np.empty((B, n), np.float32)
    ref = np.empty((B, n), np.float32)
    near = np.empty((B, n), np.float32)
    for b in range(B):
        mic[b], ref[b], near[b] = scene(n, seed0 + b, double_talk=double_talk)
    return mic, ref, near
