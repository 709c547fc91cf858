"""GPU parity: the gfx950 path (through the C ABI via Little_net) against the
reference golden vectors and the CPU oracle.  Tolerances (north_star):
integer framing bit-exact; float waveform <= 1e-4 RMS; intermediates <= 1e-5
relative."""
import json
import os

import numpy as np
import pytest
import torch

import aec_oracle as O
from conftest import CASES, GOLDEN, golden_case

pytestmark = pytest.mark.gpu

WAVE_RMS_TOL = 1e-4


def _run(net, erb, mic, ref, near, dev='cuda:0'):
    T = lambda a: torch.as_tensor(a, device=dev)[None] if a is not None else None
    erb_t = torch.tensor(erb, dtype=torch.float32, device=dev)
    with torch.no_grad():
        out, loss = net(T(mic), T(ref), T(near), erb_t)
    torch.cuda.synchronize()
    return out[0].cpu().numpy(), (float(loss) if loss is not None else None)


def _loss_ok(got, exp, tol=1e-4):
    """Loss parity; an all-zero near signal makes the reference's normaliser
    0/0 = NaN (ERB.py:256) and the loss NaN — both paths must then agree on NaN."""
    if np.isnan(exp):
        return bool(np.isnan(got))
    return abs(got - exp) <= tol * max(1.0, abs(exp))


def _rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - b) ** 2))) if np.size(a) else 0.0


@pytest.mark.parametrize('name', CASES)
def test_golden_cases(gpu_net, golden_erb, name):
    d = golden_case(name)
    out, loss = _run(gpu_net, golden_erb, d['mic'], d['ref'], d['near'])
    assert out.shape == d['out'].shape                       # bit-exact framing
    assert _rms(out, d['out']) <= WAVE_RMS_TOL
    assert abs(loss - float(d['loss'])) <= 1e-4 * max(1.0, abs(float(d['loss'])))


@pytest.mark.parametrize('name', ['case_513_3', 'case_16123_5'])
def test_intermediates(gpu_net, golden_erb, name):
    d = golden_case(name)
    gpu_net.set_debug(True)
    try:
        _run(gpu_net, golden_erb, d['mic'], d['ref'], d['near'])
        T = d['gru_out'].shape[0]
        got = {k: gpu_net.debug_intermediate(k, 1, T)[0].cpu().numpy()
               for k in ['mic_erb', 'ref_erb', 'near_erb', 'gru_out', 'mask', 'est_erb']}
    finally:
        gpu_net.set_debug(False)
    mic_erb = d['gru_in'][:, :32]
    scale = np.abs(mic_erb).max()
    assert np.abs(got['mic_erb'] - mic_erb).max() <= 1e-5 * scale
    assert np.abs(np.abs(got['mic_erb'] - got['ref_erb']) - d['gru_in'][:, 32:]).max() <= 1e-5 * scale
    assert np.abs(got['gru_out'] - d['gru_out']).max() <= 1e-5
    assert np.abs(got['mask'] - d['mask']).max() <= 1e-5
    assert np.abs(got['est_erb'] - d['mask'] * mic_erb).max() <= 1e-5 * scale


def test_long_utterance_vs_golden(gpu_net, golden_erb):
    from aec_amd import synth
    g = dict(np.load(os.path.join(GOLDEN, 'long_160000_7.npz')))
    mic, ref, near = synth.scene(160000, 7)
    out, loss = _run(gpu_net, golden_erb, mic, ref, near)
    assert out.shape[0] == int(g['out_len'])
    assert _rms(out[:2048], g['head']) <= WAVE_RMS_TOL
    assert _rms(out[-2048:], g['tail']) <= WAVE_RMS_TOL
    assert abs(np.sqrt(np.mean(out.astype(np.float64) ** 2)) - float(g['rms'])) <= 1e-4
    assert abs(loss - float(g['loss'])) <= 1e-4 * abs(float(g['loss']))


def test_ragged_batch_equals_batch_of_one(gpu_net, golden_erb):
    """One batched call with per-stream lengths == the reference run one
    utterance at a time (scripts/test.py:139 batch_size=1)."""
    from aec_amd import synth
    g = dict(np.load(os.path.join(GOLDEN, 'ragged.npz')))
    lens = [int(n) for n in g['lens']]
    L = max(lens)
    mics, refs, nears = [np.zeros((3, L), np.float32) for _ in range(3)]
    for i, n in enumerate(lens):
        mics[i, :n], refs[i, :n], nears[i, :n] = synth.scene(n, 100 + i)
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    with torch.no_grad():
        out, loss = gpu_net.forward_ragged(torch.tensor(mics, device=dev), torch.tensor(refs, device=dev),
                                           torch.tensor(nears, device=dev), erb_t, lens)
    out = out.cpu().numpy()
    assert out.shape == (3, 256 * (L // 256))
    for i, n in enumerate(lens):
        ol = 256 * (n // 256)
        assert _rms(out[i, :ol], g[f'out{i}']) <= WAVE_RMS_TOL
        assert not out[i, ol:].any()


def test_batch_invariance_and_determinism(gpu_net, golden_erb):
    """Stream b's output does not depend on the other streams (bit-exact), and
    repeated calls are bit-identical.  The 8-stream calls run the analysis as
    one (item, signal) task per wave; the 72-stream call as persistent waves
    walking items signal by signal (analysis_kernel<false>): the same bits."""
    from aec_amd import synth
    B, n = 8, 20000
    mic, ref, near = synth.batch(B, n, seed0=40)
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    M, R, N = (torch.tensor(a, device=dev) for a in (mic, ref, near))
    with torch.no_grad():
        o1, _ = gpu_net.forward_ragged(M, R, N, erb_t, [n] * B)
        o2, _ = gpu_net.forward_ragged(M, R, N, erb_t, [n] * B)
        perm = torch.tensor([3, 1, 7, 0, 2, 6, 5, 4], device=dev)
        o3, _ = gpu_net.forward_ragged(M[perm], R[perm], N[perm], erb_t, [n] * B)
        o4, _ = gpu_net.forward_ragged(M[2:3], R[2:3], N[2:3], erb_t, [n])
        rep = lambda x: x.repeat(9, 1)                               # 72 x 20 items x 3 signals > one wave round
        o5, _ = gpu_net.forward_ragged(rep(M), rep(R), rep(N), erb_t, [n] * 9 * B)
    assert torch.equal(o1, o2)
    assert torch.equal(o1[perm], o3)
    assert torch.equal(o1[2:3], o4)
    assert torch.equal(o5, rep(o1))


@pytest.mark.parametrize('n', [1000, 4097, 33333])
def test_vs_oracle_random_lengths(gpu_net, golden_weights, golden_erb, n):
    from aec_amd import synth
    mic, ref, near = synth.scene(n, 1000 + n)
    out, loss = _run(gpu_net, golden_erb, mic, ref, near)
    o, l = O.little_net_forward(mic, ref, near, golden_erb.astype(np.float32), golden_weights)
    assert out.shape == o.shape
    assert _rms(out, o) <= WAVE_RMS_TOL
    assert _loss_ok(loss, l)


def test_near_none_and_unaligned_rows(gpu_net, golden_weights, golden_erb):
    """near=None skips the loss; odd row strides (unaligned float4) take the
    scalar load path and give the same waveform."""
    from aec_amd import synth
    B, n = 3, 9001
    mic, ref, near = synth.batch(B, n, seed0=77)
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    with torch.no_grad():
        o_a, l_a = gpu_net.forward_ragged(torch.tensor(mic, device=dev), torch.tensor(ref, device=dev),
                                          None, erb_t, [n] * B)
        assert l_a is None
        # rows with stride n+3 (not a multiple of 4) via a sliced wider buffer
        wide = lambda a: torch.tensor(np.pad(a, ((0, 0), (1, 2))), device=dev)[:, 1:1 + n]
        o_b, l_b = gpu_net.forward_ragged(wide(mic), wide(ref), wide(near), erb_t, [n] * B)
    assert torch.allclose(o_a, o_b, rtol=0, atol=1e-6)
    for b in range(B):
        o, l = O.little_net_forward(mic[b], ref[b], near[b], golden_erb.astype(np.float32), golden_weights)
        assert _rms(o_b[b].cpu().numpy(), o) <= WAVE_RMS_TOL
        assert _loss_ok(float(l_b[b]), l)


def test_erle_delta_vs_oracle(gpu_net, golden_weights, golden_erb):
    """ERLE of the GPU path vs the reference-path restatement
    on far-end single talk: |delta| <= 0.1 dB."""
    from aec_amd import synth
    mic, ref, near = synth.scene(48000, 5, double_talk=False)
    near = near + np.float32(1e-3) * np.random.default_rng(5).standard_normal(48000).astype(np.float32)
    out, _ = _run(gpu_net, golden_erb, mic, ref, near)
    o, _ = O.little_net_forward(mic, ref, near, golden_erb.astype(np.float32), golden_weights)
    assert abs(O.erle_db(mic, out) - O.erle_db(mic, o)) <= 0.1


def test_unequal_signal_lengths_vs_golden(gpu_net, golden_erb):
    """aec_process_siglens: mic / ref / near at their own stored lengths
    (test.py:139 default collate) against the reference's outputs, batched
    in one ragged call; a frame-count mismatch raises like the reference."""
    d = dict(np.load(os.path.join(GOLDEN, 'siglens.npz')))
    meta = json.load(open(os.path.join(GOLDEN, 'siglens_meta.json')))
    cases = meta['cases']
    B = len(cases)
    L = max(max(c['n_mic'], c['n_ref'], c['n_near']) for c in cases)
    rows = {k: np.zeros((B, L), np.float32) for k in ('mic', 'ref', 'near')}
    lens = np.zeros((B, 3), np.int64)
    for i, c in enumerate(cases):
        for j, k in enumerate(('mic', 'ref', 'near')):
            x = d[f'{k}{i}']
            rows[k][i, :len(x)] = x
            lens[i, j] = len(x)
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    T = lambda a: torch.from_numpy(a).to(dev)
    with torch.no_grad():
        out, loss = gpu_net.forward_ragged(T(rows['mic']), T(rows['ref']), T(rows['near']), erb_t, lens)
    torch.cuda.synchronize()
    out, loss = out.cpu().numpy(), loss.cpu().numpy()
    for i, c in enumerate(cases):
        exp = d[f'out{i}']
        assert exp.shape == (c['out_len'],)
        assert _rms(out[i, :c['out_len']], exp) <= WAVE_RMS_TOL
        assert not out[i, c['out_len']:].any()
        assert _loss_ok(float(loss[i]), float(d[f'loss{i}']))
    bad = lens.copy()
    bad[1, 1] = 256 * (lens[1, 0] // 256 + 1) + 40     # ref one frame longer than mic
    assert bad[1, 1] <= L
    with pytest.raises(RuntimeError):
        gpu_net.forward_ragged(T(rows['mic']), T(rows['ref']), T(rows['near']), erb_t, bad)
    h, _ = gpu_net._handle(torch.device(dev))          # the C ABI refuses it too (AEC_ERR_INVALID_ARG)
    m, r, nn_ = T(rows['mic']), T(rows['ref']), T(rows['near'])
    o = torch.empty(B, L, device=dev)
    with pytest.raises(RuntimeError, match='frame count'):
        h.process(m.data_ptr(), r.data_ptr(), nn_.data_ptr(), bad, B, L, o.data_ptr(), L, None,
                  torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize('lens', [[33333, 4097, 255, 16000, 256], [160000]])
def test_bypass_fused_synthesis_bit_exact(golden_weights, golden_erb, monkeypatch, lens):
    """The bypass path (no NLMS: the reference-parity drop-in) with up to half
    the CUs of streams runs the GRU and the synthesis as one kernel over K2's
    packed mic rows (gru_synth_kernel, one stream per block) instead of
    gru_kernel + synthesis_kernel re-deriving the mic spectrum
    (AEC_FUSED_SYNTH=0): the same values, so the waveform and est_erb are
    bit-identical and the loss equal to summation order (<= 1e-6)."""
    import aec_amd
    from aec_amd import synth
    from conftest import PARAM_KEYS
    L = max(lens)
    mic, ref, near = (np.zeros((len(lens), L), np.float32) for _ in range(3))
    for i, n in enumerate(lens):
        mic[i, :n], ref[i, :n], near[i, :n] = synth.scene(n, 1300 + i)
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    M, R, N = (torch.tensor(a, device=dev) for a in (mic, ref, near))
    res = {}
    for fused in ('0', '1'):
        monkeypatch.setenv('AEC_FUSED_SYNTH', fused)              # read when the handle is created
        net = aec_amd.Little_net(aec_amd.speech_conf, 32).eval()
        sd = net.state_dict()
        for k in PARAM_KEYS:
            sd[k] = torch.from_numpy(golden_weights[k])
        net.load_state_dict(sd, strict=True)
        net = net.to(dev)
        net.set_debug(True)
        with torch.no_grad():
            out, loss = net.forward_ragged(M, R, N, erb_t, lens)
        est = net.debug_intermediate('est_erb', len(lens), L // 256 + 1)
        torch.cuda.synchronize()
        res[fused] = out.cpu().numpy(), loss.cpu().numpy(), est.cpu().numpy()
    (o0, l0, e0), (o1, l1, e1) = res['0'], res['1']
    assert np.array_equal(o0, o1)
    for i, n in enumerate(lens):
        assert np.array_equal(e0[i, :n // 256 + 1], e1[i, :n // 256 + 1]), i
    np.testing.assert_allclose(l1, l0, rtol=1e-6)
    if len(lens) == 1:
        o, l = O.little_net_forward(mic[0], ref[0], near[0], golden_erb.astype(np.float32), golden_weights)
        assert _rms(o1[0], o) <= WAVE_RMS_TOL
