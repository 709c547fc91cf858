"""Pin the CPU oracle (oracle/aec_oracle.py) against the reference's own
outputs (tests/golden/*, made by tests/golden/make_golden.py from
/root/reference).  CPU only."""
import hashlib
import json
import os

import numpy as np
import pytest

import aec_oracle as O
from conftest import CASES, GOLDEN, golden_case


def test_framing_integers():
    for n, T, L in [(255, 1, 0), (256, 2, 256), (511, 2, 256), (512, 3, 512), (513, 3, 512),
                    (16000, 63, 15872), (16123, 63, 15872), (160000, 626, 160000), (159999, 625, 159744)]:
        assert O.n_frames(n) == T
        assert O.out_len(n) == L


def test_erb_filterbank_matches_reference(golden_erb):
    e = O.erb_filters()
    assert e.shape == (257, 32)
    assert np.array_equal(e, golden_erb)            # float64 bit-exact
    assert int((golden_erb != 0).sum()) == 483
    assert not golden_erb[0].any() and not golden_erb[256].any()   # DC / Nyquist uncovered


def test_stft_bases_closed_form(golden_weights):
    """The reference's conv bases are exactly the windowed rDFT / irDFT."""
    w = golden_weights
    n = np.arange(512)
    win = O.hann()
    assert np.abs(w['istft_window'] - win).max() < 1e-7
    for r, fwd, inv in zip(w['stft_rows'], w['stft_weight_rows'], w['istft_weight_rows']):
        k = r if r < 257 else r - 257
        base = np.cos(2 * np.pi * k * n / 512) if r < 257 else -np.sin(2 * np.pi * k * n / 512)
        assert np.abs(base * win - fwd).max() < 1e-6
        ck = 1.0 if k in (0, 256) else 2.0
        exp = base * win * ck / 512
        assert np.abs(exp - inv).max() < 1e-7


@pytest.mark.parametrize('name', CASES)
def test_oracle_vs_reference_golden(name, golden_weights, golden_erb):
    d = golden_case(name)
    out, loss, I = O.little_net_forward(d['mic'], d['ref'], d['near'], golden_erb.astype(np.float32),
                                        golden_weights, return_intermediates=True)
    assert out.shape == d['out'].shape                              # bit-exact framing
    if out.size:
        rms = np.sqrt(np.mean((out - d['out']) ** 2))
        assert rms < 5e-6, rms
    assert abs(loss - float(d['loss'])) < 1e-5 * max(1, abs(loss))
    assert np.abs(I['gru_in'] - d['gru_in']).max() < 1e-4 * max(1, np.abs(d['gru_in']).max())
    assert np.abs(I['gru_out'] - d['gru_out']).max() < 1e-5
    assert np.abs(I['mask'] - d['mask']).max() < 1e-5
    if 'mic_spec' in d:
        ms = d['mic_spec']
        S = O.stft(O.normalise(d['mic']))
        assert np.abs(S.real.T - ms[:257]).max() < 1e-4
        assert np.abs(S.imag.T - ms[257:]).max() < 1e-4


def test_long_case_inputs_regenerate():
    """The 10 s golden keeps only a summary; its inputs must regenerate bit-exactly."""
    from aec_amd import synth
    meta = json.load(open(os.path.join(GOLDEN, 'golden_meta.json')))['long_160000_7']
    mic, ref, near = synth.scene(meta['n'], meta['seed'])
    h = hashlib.sha256(mic.tobytes() + ref.tobytes() + near.tobytes()).hexdigest()
    assert h == meta['input_sha256']


def test_long_case_oracle(golden_weights, golden_erb):
    from aec_amd import synth
    g = dict(np.load(os.path.join(GOLDEN, 'long_160000_7.npz')))
    mic, ref, near = synth.scene(160000, 7)
    out, loss = O.little_net_forward(mic, ref, near, golden_erb.astype(np.float32), golden_weights)
    assert out.shape[0] == int(g["out_len"]) == 160000
    assert np.sqrt(np.mean((out[:2048] - g['head']) ** 2)) < 5e-6
    assert np.sqrt(np.mean((out[-2048:] - g['tail']) ** 2)) < 5e-6
    assert abs(np.sqrt(np.mean(out ** 2)) - float(g['rms'])) < 1e-5
    assert abs(loss - float(g['loss'])) < 1e-5 * abs(loss)


def test_ragged_per_utterance(golden_weights, golden_erb):
    from aec_amd import synth
    g = dict(np.load(os.path.join(GOLDEN, 'ragged.npz')))
    for i, n in enumerate(g['lens']):
        mic, ref, near = synth.scene(int(n), 100 + i)
        out, loss = O.little_net_forward(mic, ref, near, golden_erb.astype(np.float32), golden_weights)
        assert out.shape == g[f'out{i}'].shape
        assert np.sqrt(np.mean((out - g[f'out{i}']) ** 2)) < 5e-6


def test_nlms_known_answers():
    """Build-defined FD-NLMS (parity unpinned vs the reference): mu = 0 is the
    identity on the mic spectrum; on a pure echo path it converges."""
    from aec_amd import synth
    mic, ref, near = synth.scene(48000, 11, double_talk=False)
    Sm, Sr = O.stft(O.normalise(mic)), O.stft(O.normalise(ref))
    E0 = O.nlms(Sm, Sr, taps=4, mu=0.0)
    assert np.array_equal(E0, Sm)
    E = O.nlms(Sm, Sr, taps=4, mu=0.3)
    T = Sm.shape[0]
    tail = slice(T // 2, T)
    erle = 10 * np.log10(np.sum(np.abs(Sm[tail]) ** 2) / np.sum(np.abs(E[tail]) ** 2))
    assert erle > 5.0, erle


def test_torch_port_matches_golden(golden_weights, golden_erb):
    """The CPU-baseline port (bench.py cpu_baseline) reproduces the reference."""
    import torch
    from torch_port import TorchPort
    port = TorchPort(golden_weights, golden_erb)
    for name in ['case_513_3', 'case_16123_5']:
        d = golden_case(name)
        out, loss = port(*(torch.from_numpy(d[k])[None] for k in ('mic', 'ref', 'near')))
        assert out.shape[1] == d['out'].shape[0]
        assert np.sqrt(np.mean((out[0].numpy() - d['out']) ** 2)) < 1e-5
        assert abs(float(loss[0]) - float(d['loss'])) < 1e-5 * abs(float(d['loss']))


def test_oracle_vs_reference_unequal_signal_lengths(golden_weights, golden_erb):
    """test.py:139 feeds each signal at its stored length (default collate):
    the oracle's per-signal normaliser / framing reproduces the reference on
    unequal lengths with equal frame counts (tests/golden/make_siglens_golden.py)."""
    d = dict(np.load(os.path.join(GOLDEN, 'siglens.npz')))
    meta = json.load(open(os.path.join(GOLDEN, 'siglens_meta.json')))
    assert meta['mismatch'] == 'RuntimeError'                     # the reference raises on a frame mismatch
    for i, c in enumerate(meta['cases']):
        mic, ref, near = d[f'mic{i}'], d[f'ref{i}'], d[f'near{i}']
        assert (len(mic), len(ref), len(near)) == (c['n_mic'], c['n_ref'], c['n_near'])
        out, loss = O.little_net_forward(mic, ref, near, golden_erb.astype(np.float32), golden_weights)
        assert out.shape == d[f'out{i}'].shape == (c['out_len'],)
        assert np.sqrt(np.mean((out - d[f'out{i}']) ** 2)) < 5e-6
        assert abs(loss - float(d[f'loss{i}'])) < 1e-5 * max(1, abs(loss))
    with pytest.raises(ValueError):                               # numpy's shape error, as torch's RuntimeError
        O.little_net_forward(mic[:3000], ref[:3300], near[:3000], golden_erb, golden_weights)
