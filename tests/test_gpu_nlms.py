"""GPU parity of the FD-NLMS stage.

The reference has no linear echo canceller, so the float64 restatement
oracle/aec_oracle.py:nlms / aec_forward is the only oracle ("parity unpinned"
against the reference itself); its known answers are pinned in
tests/test_oracle_golden.py.  Here the gfx950 path (C ABI via Little_net with
``nlms=``) is held to the same bars as the bypass path: integer framing
bit-exact, waveform <= 1e-4 RMS, features <= 1e-5 relative, ERLE delta <= 0.1 dB.
"""
import numpy as np
import pytest
import torch

import aec_oracle as O
from conftest import PARAM_KEYS

pytestmark = pytest.mark.gpu

WAVE_RMS_TOL = 1e-4
NLMS = dict(taps=4, mu=0.3, beta=0.5, delta=1e-4)      # aec_amd.configs.nlms_conf


def _net(golden_weights, nlms):
    import aec_amd
    net = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=nlms).eval()
    sd = net.state_dict()
    for k in PARAM_KEYS:
        sd[k] = torch.from_numpy(golden_weights[k])
    net.load_state_dict(sd, strict=True)
    return net.to('cuda:0')


@pytest.fixture(scope='module')
def nlms_net(golden_weights):
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    return _net(golden_weights, NLMS)


def _rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - b) ** 2))) if np.size(a) else 0.0


def _loss_ok(got, exp, tol=1e-4):
    if np.isnan(exp):
        return bool(np.isnan(got))
    return abs(got - exp) <= tol * max(1.0, abs(exp))


def _run(net, erb, mic, ref, near):
    dev = 'cuda:0'
    T = lambda a: torch.as_tensor(a, device=dev)[None] if a is not None else None
    with torch.no_grad():
        out, loss = net(T(mic), T(ref), T(near), torch.tensor(erb, dtype=torch.float32, device=dev))
    torch.cuda.synchronize()
    return out[0].cpu().numpy(), (float(loss) if loss is not None else None)


@pytest.mark.parametrize('n', [255, 256, 513, 4097, 16123, 33333])
def test_nlms_vs_oracle(nlms_net, golden_weights, golden_erb, n):
    from aec_amd import synth
    mic, ref, near = synth.scene(n, 2000 + n)
    out, loss = _run(nlms_net, golden_erb, mic, ref, near)
    o, l = O.aec_forward(mic, ref, near, golden_erb.astype(np.float32), golden_weights, nlms_cfg=NLMS)
    assert out.shape == o.shape                               # bit-exact framing
    assert _rms(out, o) <= WAVE_RMS_TOL
    assert _loss_ok(loss, l)


def test_nlms_features_vs_oracle(nlms_net, golden_erb):
    """mic_erb = ERB(|E|) of the NLMS error, ref_erb / near_erb unchanged."""
    from aec_amd import synth
    n = 20000
    mic, ref, near = synth.scene(n, 31)
    erb = golden_erb.astype(np.float32).astype(np.float64)
    nlms_net.set_debug(True)
    try:
        _run(nlms_net, golden_erb, mic, ref, near)
        T = n // 256 + 1
        got = {k: nlms_net.debug_intermediate(k, 1, T)[0].cpu().numpy() for k in ['mic_erb', 'ref_erb', 'near_erb']}
    finally:
        nlms_net.set_debug(False)
    Sm, Sr, Sn = (O.stft(O.normalise(x)) for x in (mic, ref, near))
    E = O.nlms(Sm, Sr, **NLMS)
    exp = {'mic_erb': O.magnitude(E) @ erb, 'ref_erb': O.magnitude(Sr) @ erb, 'near_erb': O.magnitude(Sn) @ erb}
    for k in exp:
        scale = np.abs(exp[k]).max()
        assert np.abs(got[k] - exp[k]).max() <= 1e-5 * scale, k


@pytest.mark.parametrize('taps', [1, 2, 8])
def test_nlms_tap_counts(golden_weights, golden_erb, taps):
    from aec_amd import synth
    cfg = dict(NLMS, taps=taps)
    net = _net(golden_weights, cfg)
    mic, ref, near = synth.scene(12345, 50 + taps)
    out, loss = _run(net, golden_erb, mic, ref, near)
    o, l = O.aec_forward(mic, ref, near, golden_erb.astype(np.float32), golden_weights, nlms_cfg=cfg)
    assert _rms(out, o) <= WAVE_RMS_TOL
    assert _loss_ok(loss, l)


def test_nlms_mu0_equals_bypass(golden_weights, golden_erb, gpu_net):
    """Known answer: mu = 0 keeps W = 0, so E = D exactly and the path equals
    the reference-parity bypass.  The two paths run the same transform in
    different kernels (the compiler may contract differently), so equality
    is to float32 rounding: <= 1e-6 of the signal scale."""
    from aec_amd import synth
    net0 = _net(golden_weights, dict(NLMS, mu=0.0))
    B, n = 4, 17000
    mic, ref, near = synth.batch(B, n, seed0=90)
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    M, R, N = (torch.tensor(a, device=dev) for a in (mic, ref, near))
    with torch.no_grad():
        a, la = net0.forward_ragged(M, R, N, erb_t, [n] * B)
        b, lb = gpu_net.forward_ragged(M, R, N, erb_t, [n] * B)
    assert float((a - b).abs().max()) <= 1e-6 * float(b.abs().max())
    # an all-zero near row gives the reference's NaN loss (0/0 normaliser) on both paths
    torch.testing.assert_close(la, lb, rtol=1e-6, atol=0.0, equal_nan=True)


def test_nlms_ragged_and_batch_invariance(nlms_net, golden_weights, golden_erb):
    from aec_amd import synth
    lens = [7000, 12801, 9472, 300]
    L = max(lens)
    rows = [synth.scene(n, 600 + i) for i, n in enumerate(lens)]
    mic, ref, near = (np.zeros((len(lens), L), np.float32) for _ in range(3))
    for i, (m, r, nn_) in enumerate(rows):
        mic[i, :lens[i]], ref[i, :lens[i]], near[i, :lens[i]] = m, r, nn_
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    M, R, N = (torch.tensor(a, device=dev) for a in (mic, ref, near))
    with torch.no_grad():
        out, loss = nlms_net.forward_ragged(M, R, N, erb_t, lens)
        out2, _ = nlms_net.forward_ragged(M[1:2], R[1:2], N[1:2], erb_t, lens[1:2])
    out = out.cpu().numpy()
    for i, n in enumerate(lens):
        ol = 256 * (n // 256)
        o, l = O.aec_forward(*rows[i], golden_erb.astype(np.float32), golden_weights, nlms_cfg=NLMS)
        assert _rms(out[i, :ol], o) <= WAVE_RMS_TOL
        assert not out[i, ol:].any()
        assert _loss_ok(float(loss[i]), l)
    assert np.array_equal(out[1:2, :out2.shape[1]], out2.cpu().numpy())


def test_nlms_erle_delta_vs_oracle(nlms_net, golden_weights, golden_erb):
    from aec_amd import synth
    mic, ref, near = synth.scene(48000, 9, double_talk=False)
    near = near + np.float32(1e-3) * np.random.default_rng(9).standard_normal(48000).astype(np.float32)
    out, _ = _run(nlms_net, golden_erb, mic, ref, near)
    o, _ = O.aec_forward(mic, ref, near, golden_erb.astype(np.float32), golden_weights, nlms_cfg=NLMS)
    assert abs(O.erle_db(mic, out) - O.erle_db(mic, o)) <= 0.1


def test_fused_synthesis_bit_exact(golden_weights, golden_erb, monkeypatch):
    """The fused GRU + synthesis kernel (aec_gru_synth.hip, default on the
    NLMS path) against the separate gru_kernel + synthesis_kernel
    (AEC_FUSED_SYNTH=0), with one and with two streams per fused block
    (AEC_GRU_NS; B = 5 leaves the last block one stream): the same per-sample
    arithmetic, so the waveform and est_erb are bit-identical; the loss is
    summed in a different order (<= 1e-6 relative).  Ragged lengths cover
    partial last chunks and a stream shorter than one chunk."""
    from aec_amd import synth
    lens = [33333, 4097, 255, 16000, 256]
    L = max(lens)
    rows = [synth.scene(n, 700 + i) for i, n in enumerate(lens)]
    mic, ref, near = (np.zeros((len(lens), L), np.float32) for _ in range(3))
    for i, (m, r, nn_) in enumerate(rows):
        mic[i, :lens[i]], ref[i, :lens[i]], near[i, :lens[i]] = m, r, nn_
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    M, R, N = (torch.tensor(a, device=dev) for a in (mic, ref, near))
    res = {}
    # NS = 1: overlap-add on the head waves; NS = 2: on the recurrence waves (aec_gru_synth.hip)
    for fused, ns in (('0', '2'), ('1', '1'), ('1', '2')):
        monkeypatch.setenv('AEC_FUSED_SYNTH', fused)             # read when the handle is created
        monkeypatch.setenv('AEC_GRU_NS', ns)                    # streams per fused block, read per launch
        net = _net(golden_weights, NLMS)
        net.set_debug(True)
        with torch.no_grad():
            out, loss = net.forward_ragged(M, R, N, erb_t, lens)
        est = net.debug_intermediate('est_erb', len(lens), L // 256 + 1)
        torch.cuda.synchronize()
        res[fused + ns] = (out.cpu().numpy(), loss.cpu().numpy(), est.cpu().numpy())
    o0, l0, e0 = res['02']
    for key in ('11', '12'):                                     # one and two streams per block (B = 5: odd)
        o1, l1, e1 = res[key]
        assert np.array_equal(o0, o1), key
        for i, n in enumerate(lens):
            assert np.array_equal(e0[i, :n // 256 + 1], e1[i, :n // 256 + 1]), (key, i)
        np.testing.assert_allclose(l1, l0, rtol=1e-6)


def test_small_batch_split_path_bit_exact(golden_weights, golden_erb, monkeypatch):
    """Few streams take the split NLMS path (frame-parallel transforms + rows,
    per-stream recursion, frame-parallel mic_erb; AEC_SMALLB) instead of the
    per-stream K2n block: the same per-frame arithmetic, so the waveform,
    the features and the loss are bit-identical to the K2n path; so is K2n
    with the ref waves' two ERB projections in two passes (AEC_NLMS_MODE
    bit 4) instead of the merged pass."""
    from aec_amd import synth
    lens = [33333, 4097, 255, 16000, 256]
    L = max(lens)
    rows = [synth.scene(n, 800 + i) for i, n in enumerate(lens)]
    mic, ref, near = (np.zeros((len(lens), L), np.float32) for _ in range(3))
    for i, (m, r, nn_) in enumerate(rows):
        mic[i, :lens[i]], ref[i, :lens[i]], near[i, :lens[i]] = m, r, nn_
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    M, R, N = (torch.tensor(a, device=dev) for a in (mic, ref, near))
    res = {}
    for small in ('0', '64', '0m'):
        monkeypatch.setenv('AEC_SMALLB', small.rstrip('m'))     # read when the handle is created
        monkeypatch.setenv('AEC_NLMS_MODE', '16' if small == '0m' else '0')
        net = _net(golden_weights, NLMS)
        net.set_debug(True)
        with torch.no_grad():
            out, loss = net.forward_ragged(M, R, N, erb_t, lens)
        T = L // 256 + 1
        feats = {k: net.debug_intermediate(k, len(lens), T).cpu().numpy() for k in ('mic_erb', 'ref_erb', 'est_erb')}
        torch.cuda.synchronize()
        res[small] = (out.cpu().numpy(), loss.cpu().numpy(), feats)
    o0, l0, f0 = res['0']
    for key in ('64', '0m'):
        o1, l1, f1 = res[key]
        assert np.array_equal(o0, o1), key
        assert np.array_equal(l0, l1, equal_nan=True), key   # the 256-sample row's loss is the reference's 0/0 NaN
        for k in f0:
            for i, n in enumerate(lens):
                assert np.array_equal(f0[k][i, :n // 256 + 1], f1[k][i, :n // 256 + 1], equal_nan=True), (key, k, i)


@pytest.mark.parametrize('B,n', [(5, 0), (1, 160000), (64, 160000), (128, 48000)])
def test_small_batch_pipeline_bit_exact(golden_weights, golden_erb, monkeypatch, B, n):
    """The pipelined split path (AEC_SMALLB_PIPE, default on): the NLMS
    recursion and mic_erb run in producer blocks of the GRU + synthesis launch,
    one 16-frame chunk ahead of the consumer block of the same stream (spin
    waits on a per-stream counter, sc1 hand-off).  Waveform, mic_erb / ref_erb /
    est_erb and loss are bit-identical to the three-launch split path
    (AEC_SMALLB_PIPE=0) and the waveform to the per-stream K2n block
    (AEC_SMALLB=0): ragged lengths (n = 0: 33333, 4097, 255, 16000, 256), one
    10 s stream (the batch-1 latency case), 64 of them (128 blocks spread
    over every XCD) and 128 streams of 3 s (256 blocks: one per CU, the
    path's limit).  Repeated calls reuse the counters (a new epoch per call)."""
    from aec_amd import synth
    if n == 0:
        lens = [33333, 4097, 255, 16000, 256]
        rows = [synth.scene(m, 900 + i) for i, m in enumerate(lens)]
        L = max(lens)
        mic, ref, near = (np.zeros((B, L), np.float32) for _ in range(3))
        for i, (m, r, nn_) in enumerate(rows):
            mic[i, :lens[i]], ref[i, :lens[i]], near[i, :lens[i]] = m, r, nn_
    else:
        lens = [n] * B
        L = n
        mic, ref, near = synth.batch(B, n, seed0=950)
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    M, R, N = (torch.tensor(a, device=dev) for a in (mic, ref, near))
    T = L // 256 + 1
    res = {}
    for key, env in (('pipe', {'AEC_SMALLB_PIPE': '1'}), ('split', {'AEC_SMALLB_PIPE': '0'}),
                     ('k2n', {'AEC_SMALLB': '0'})):
        for k in ('AEC_SMALLB_PIPE', 'AEC_SMALLB'):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)                               # read when the handle is created
        net = _net(golden_weights, NLMS)
        net.set_debug(True)
        with torch.no_grad():
            outs = [net.forward_ragged(M, R, N, erb_t, lens) for _ in range(2 if key == 'pipe' else 1)]
        feats = {k: net.debug_intermediate(k, B, T).cpu().numpy() for k in ('mic_erb', 'ref_erb', 'est_erb')}
        torch.cuda.synchronize()
        res[key] = [(o.cpu().numpy(), l.cpu().numpy()) for o, l in outs], feats
    (o0, l0), (o0b, l0b) = res['pipe'][0]
    assert np.array_equal(o0, o0b) and np.array_equal(l0, l0b, equal_nan=True)   # second epoch
    f0 = res['pipe'][1]
    (o1, l1), = res['split'][0]
    assert np.array_equal(o0, o1)
    assert np.array_equal(l0, l1, equal_nan=True)
    for k in f0:
        for i, m in enumerate(lens):
            assert np.array_equal(f0[k][i, :m // 256 + 1], res['split'][1][k][i, :m // 256 + 1], equal_nan=True), (k, i)
    (o2, _), = res['k2n'][0]
    assert np.array_equal(o0, o2)
    if n:
        o, l = O.aec_forward(mic[0], ref[0], near[0], golden_erb.astype(np.float32), golden_weights, nlms_cfg=NLMS)
        assert _rms(o0[0], o) <= WAVE_RMS_TOL
        assert _loss_ok(float(l0[0]), l)


def test_small_batch_pipeline_timeout_reported(golden_weights, golden_erb, monkeypatch):
    """The pipeline's spin waits are bounded: with the producers made silent
    (AEC_SMALLB_PIPE_STALL=N, read per call: nothing is published and every
    consumer wave gives up after N polls) the launch still drains, the
    handle's next call fails loudly (the timed-out call's output is invalid),
    and the call after that is bit-identical to a fresh handle."""
    from aec_amd import synth
    B, n = 3, 20000
    mic, ref, near = synth.batch(B, n, seed0=970)
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    M, R, N = (torch.tensor(a, device=dev) for a in (mic, ref, near))
    net = _net(golden_weights, NLMS)
    with torch.no_grad():
        monkeypatch.setenv('AEC_SMALLB_PIPE_STALL', '64')
        net.forward_ragged(M, R, N, erb_t, [n] * B)
        torch.cuda.synchronize()
        monkeypatch.delenv('AEC_SMALLB_PIPE_STALL')
        with pytest.raises(RuntimeError, match='timed out waiting for its producer'):
            net.forward_ragged(M, R, N, erb_t, [n] * B)
        out, loss = net.forward_ragged(M, R, N, erb_t, [n] * B)
        ref_out, ref_loss = _net(golden_weights, NLMS).forward_ragged(M, R, N, erb_t, [n] * B)
    torch.cuda.synchronize()
    assert torch.equal(out, ref_out)
    assert torch.equal(loss, ref_loss)


def test_normaliser_lookahead_bit_exact(nlms_net, golden_erb):
    """aec_prepare_siglens / aec_process_prepared (Little_net.prepare_ragged ->
    forward_ragged(lookahead=token)): the normaliser pass of a batch queued on a
    side stream ahead of its forward call.  The waveform and loss are
    bit-identical to the call without look-ahead, for the batch K2n path
    (B = 140, above the split path's half-the-CUs limit) and the pipelined
    split path (B = 5), with per-signal lengths.  A token
    prepared for other lengths is refused (nothing runs); a token that is not
    pending is refused; a later token drops the older pending one; at most two
    look-aheads may be pending; and a plain forward never consumes a pending
    look-ahead, so a buffer refilled at the same address with the same lengths
    is normalised with its own statistics (no stale constants)."""
    from aec_amd import synth
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    side = torch.cuda.Stream()
    for lens in ([33333, 4097, 255, 16000, 256], [16000, 4097, 33333, 12000, 700, 256, 5000] * 20):
        L = max(lens)
        mic, ref, near = (np.zeros((len(lens), L), np.float32) for _ in range(3))
        for i, n in enumerate(lens):
            m, r, nn_ = synth.scene(n, 900 + i)
            mic[i, :n], ref[i, :n], near[i, :n] = m, r, nn_
        M, R, N = (torch.tensor(a, device=dev) for a in (mic, ref, near))
        l3 = np.array([[n, n - n % 256 + (n % 256) // 2, n] for n in lens], np.int64)   # ref shorter, same frames
        cur = torch.cuda.current_stream()
        with torch.no_grad():
            o0, s0 = nlms_net.forward_ragged(M, R, N, erb_t, l3)
            o0, s0 = o0.cpu().numpy(), s0.cpu().numpy()
            for rep in range(2):                      # the second round reuses the handle's slots
                with torch.cuda.stream(side):
                    tok = nlms_net.prepare_ragged(M, R, N, l3, producer=cur)
                assert tok > 0
                o1, s1 = nlms_net.forward_ragged(M, R, N, erb_t, l3, lookahead=tok)
                assert np.array_equal(o0, o1.cpu().numpy()), (len(lens), rep)
                assert np.array_equal(s0, s1.cpu().numpy(), equal_nan=True), (len(lens), rep)
                with pytest.raises(RuntimeError, match='not pending'):      # consumed
                    nlms_net.forward_ragged(M, R, N, erb_t, l3, lookahead=tok)
            with torch.cuda.stream(side):             # other lengths: refused, then dropped by a later token
                bad = nlms_net.prepare_ragged(M, R, N, [L] * len(lens), producer=cur)
            with pytest.raises(RuntimeError, match='other signals'):
                nlms_net.forward_ragged(M, R, N, erb_t, l3, lookahead=bad)
            with torch.cuda.stream(side):
                t1 = nlms_net.prepare_ragged(M, R, N, l3, producer=cur)
                with pytest.raises(RuntimeError):     # two pending (bad, t1)
                    nlms_net.prepare_ragged(M, R, N, l3)
            o2, _ = nlms_net.forward_ragged(M, R, N, erb_t, l3, lookahead=t1)   # drops `bad`
            assert np.array_equal(o0, o2.cpu().numpy())
            with pytest.raises(RuntimeError, match='not pending'):
                nlms_net.forward_ragged(M, R, N, erb_t, l3, lookahead=bad)
            # a pending look-ahead, then the buffers refilled in place (same pointers, same lengths):
            # the plain forward runs its own pass on the new contents
            with torch.cuda.stream(side):
                stale = nlms_net.prepare_ragged(M, R, N, l3, producer=cur)
            side.synchronize()
            M2, R2, N2 = M.clone(), R.clone(), N.clone()
            M.mul_(3.0).add_(0.01)
            R.mul_(0.5)
            ofresh, _ = nlms_net.forward_ragged(M.clone(), R.clone(), N.clone(), erb_t, l3)
            oplain, _ = nlms_net.forward_ragged(M, R, N, erb_t, l3)
            assert np.array_equal(ofresh.cpu().numpy(), oplain.cpu().numpy())
            assert not np.array_equal(oplain.cpu().numpy(), o0)
            M.copy_(M2), R.copy_(R2), N.copy_(N2)
            o3, _ = nlms_net.forward_ragged(M, R, N, erb_t, l3, lookahead=stale)   # still pending, contents restored
            assert np.array_equal(o0, o3.cpu().numpy())
        torch.cuda.synchronize()


@pytest.mark.parametrize('B', [5, 140, 256])
def test_no_near_waveform_bit_exact(nlms_net, golden_erb, B):
    """near=None (the deployment form: no clean near-end signal, no loss;
    test.py:157 keeps only out_wav): the K2n mic waves skip the near transform
    and the normaliser pass covers mic / ref only.  The waveform must be
    bit-identical to the call with near, on the pipelined split path (B = 5)
    and the batch K2n path (B = 140, the bench's B = 256), with and without a
    look-ahead normaliser token (bench.py's `no_near` leg)."""
    from aec_amd import synth
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    rng = np.random.default_rng(B)
    lens = [int(x) for x in rng.integers(256, 48000, size=B)]
    lens[0] = 48000
    L = max(lens)
    mic, ref, near = (np.zeros((B, L), np.float32) for _ in range(3))
    for i, n in enumerate(lens):
        m, r, nn_ = synth.scene(n, 1300 + i)
        mic[i, :n], ref[i, :n], near[i, :n] = m, r, nn_
    M, R, N = (torch.tensor(a, device=dev) for a in (mic, ref, near))
    side = torch.cuda.Stream()
    with torch.no_grad():
        o0, l0 = nlms_net.forward_ragged(M, R, N, erb_t, lens)
        o1, l1 = nlms_net.forward_ragged(M, R, None, erb_t, lens)
        assert l0 is not None and l1 is None
        assert np.array_equal(o0.cpu().numpy(), o1.cpu().numpy())
        with torch.cuda.stream(side):
            tok = nlms_net.prepare_ragged(M, R, None, lens, producer=torch.cuda.current_stream())
        o2, l2 = nlms_net.forward_ragged(M, R, None, erb_t, lens, lookahead=tok)
        assert l2 is None
        assert np.array_equal(o0.cpu().numpy(), o2.cpu().numpy())
    torch.cuda.synchronize()


def test_max_batch_4096_streams_matches_single_calls(nlms_net, golden_erb):
    """BASELINE C4/C5's 4,096-stream sweep point at 10 s: > 4 GiB spectrum and
    input buffers (64-bit row / spectrum offsets), ragged lengths.  Sampled
    streams of the 4,096-stream call must be bit-identical to the same
    streams run alone (batch=1 semantics, Tester.test scripts/test.py:137-169);
    the single-stream path is itself held to the oracle above."""
    B, N = 4096, 160000
    dev = 'cuda:0'
    g = torch.Generator(device=dev).manual_seed(4096)
    ref = 0.1 * torch.randn(B, N, device=dev, generator=g)
    near = 0.05 * torch.randn(B, N, device=dev, generator=g)
    mic = 0.5 * torch.roll(ref, 128, dims=1) + near + 1e-3 * torch.randn(B, N, device=dev, generator=g)
    lens = torch.randint(N // 2, N + 1, (B,), generator=torch.Generator().manual_seed(7)).tolist()
    lens[-1] = N
    lens[0] = 300
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    with torch.no_grad():
        out, loss = nlms_net.forward_ragged(mic, ref, near, erb_t, lens)
        torch.cuda.synchronize()
        assert torch.isfinite(out).all()
        for i in (0, 1, 2047, 3333, B - 1):
            o1, l1 = nlms_net.forward_ragged(mic[i:i + 1], ref[i:i + 1], near[i:i + 1], erb_t, lens[i:i + 1])
            ol = 256 * (lens[i] // 256)
            assert torch.equal(out[i, :ol], o1[0, :ol]), i
            assert not out[i, ol:].any()
            assert abs(float(loss[i]) - float(l1[0])) <= 1e-6 * max(1.0, abs(float(l1[0]))), i
    del mic, ref, near, out
    torch.cuda.empty_cache()


def test_nlms_10s_batch_vs_oracle(nlms_net, golden_weights, golden_erb):
    """BASELINE C2 lengths: 10 s streams (626 dependent NLMS frames per bin)
    through the batch path the bench runs (B above the split path's limit of
    half the CUs: one K2n block per stream, two streams per GRU block),
    checked against the float64 oracle: waveform <= 1e-4 RMS, loss <= 1e-4
    relative; the same stream alone (the pipelined split path) gives the same
    waveform bits."""
    from aec_amd import synth
    n, B = 160000, 160
    mic, ref, near = synth.batch(B, n, seed0=4400)
    dev = 'cuda:0'
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    M, R, N = (torch.from_numpy(a).to(dev) for a in (mic, ref, near))
    with torch.no_grad():
        out, loss = nlms_net.forward_ragged(M, R, N, erb_t, [n] * B)
        out1, loss1 = nlms_net.forward_ragged(M[:1], R[:1], N[:1], erb_t, [n])
    torch.cuda.synchronize()
    out, loss = out.cpu().numpy(), loss.cpu().numpy()
    for b in (0, 41, B - 1):
        o, l = O.aec_forward(mic[b], ref[b], near[b], golden_erb.astype(np.float32), golden_weights, nlms_cfg=NLMS)
        assert out[b].shape == o.shape == (n,)
        assert _rms(out[b], o) <= WAVE_RMS_TOL, b
        assert _loss_ok(float(loss[b]), l), b
    assert np.array_equal(out1[0].cpu().numpy(), out[0])
    assert float(loss1[0]) == pytest.approx(float(loss[0]), rel=1e-6)
