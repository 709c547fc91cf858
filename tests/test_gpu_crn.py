"""GPU parity of the DCCRN path (include/aec_crn.h via aec_amd.dccrn /
aec_amd.dccrn2) against the golden vectors the reference produced
(tests/golden/make_crn_golden.py) and the float64 oracle.

Tolerances (relative RMS, written here):
* f32 path (exact f32 MFMA): out_wav, out_spec, mask, near_specs <= 1e-4
  (observed float32-reference vs float64-oracle: ~6e-7);
* bf16 path (bf16 storage / MFMA, f32 accumulate): out_wav <= BF16_WAV_TOL,
  mask <= BF16_MASK_TOL (reduced precision; the f32 path is the parity gate;
  observed out_wav relative RMS vs the reference 0.0018-0.0034 on the
  goldens, so the bar is ~1.8x the observed error);
* fp8 path (bf16 + MX-fp8 GEMMs for the LSTM input projections and the
  wide conv layers, encoder 4-5 / decoder levels 5-6: e4m3 weights and
  activations, E8M0 scale per 32 k): out_wav <= FP8_WAV_TOL, mask <=
  FP8_MASK_TOL against the reference, and within FP8_VS_BF16_TOL of the bf16
  path (the only change is those GEMMs' operand rounding; observed out_wav
  relative RMS vs the reference 0.0025-0.0045);
* BASELINE config 3's own shape (256 x 10 s in one call, 626-frame
  recurrence): three rows against the reference op mix (oracle/torch_crn_port,
  f32, pinned by tests/test_crn_oracle.py) within the same bars, and ERLE
  within C3_ERLE_DB of it;
* integer framing (T, output length) bit-exact; batch composition (ragged
  rows in one call vs one call per row) bit-exact on every path.
"""
import copy
import json
import os

import numpy as np
import pytest
import torch

import aec_amd
import crn_oracle as C
from conftest import margin

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
META = json.load(open(os.path.join(GOLD, 'crn_meta.json')))
# Reduced-precision bars: ~1.5-2x the largest error observed on MI355X (round 5,
# gpurun_out/parity_margins.json -> profiles/r05a_parity_margins.json), so a change
# that doubles an error fails.  Observed maxima: bf16 out_wav 0.0034 / mask 0.0032,
# fp8 out_wav 0.0051 / mask 0.0104, fp8 vs bf16 0.0038, persistent vs step 0.00026,
# MX vs bf16 recurrence 0.0018, ERLE delta 0.0073 dB (the 0.1 dB bar is north_star's).
# The same maxima on every box of rounds 5-6 (the kernels are deterministic; toolchain:
# ROCm 7.2 hipcc / amdclang 20 for gfx950, torch 2.10.0+rocm7.0 for the CPU op-mix ports);
# the two tightest bars (fp8 mask, persistent vs step) hold >= 2x headroom.
F32_TOL = 1e-4
BF16_WAV_TOL = 6e-3
BF16_MASK_TOL = 6e-3
FP8_WAV_TOL = 1e-2
FP8_MASK_TOL = 2.1e-2
FP8_VS_BF16_TOL = 7e-3
C3_ERLE_DB = 0.1
PERSIST_TOL = 5.5e-4
MX_VS_BF16_STEP_TOL = 3.5e-3


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if b.size == 0:
        return 0.0
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-30))


def build(name, dtype):
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    m = META[name]
    conf = copy.deepcopy(aec_amd.net_conf)
    conf.update(m['overrides'])
    net = (aec_amd.dccrn if m['version'] == 1 else aec_amd.dccrn2).DCCRN(conf, dtype=dtype).eval()
    sd = net.state_dict()
    for k, v in C.make_weights(conf, m['version'], m['weight_seed']).items():
        sd[k] = torch.from_numpy(v)
    net.load_state_dict(sd, strict=True)
    return net.to('cuda:0'), m, conf


def T(a):
    return torch.as_tensor(np.asarray(a), device='cuda:0')[None]


@pytest.mark.parametrize('name', sorted(META))
def test_f32_matches_reference(name):
    net, m, _ = build(name, 'f32')
    d = np.load(os.path.join(GOLD, f'crn_{name}.npz'))
    with torch.no_grad():
        res = net(T(d['mic']), T(d['far']), T(d['near']), T(d['echo']))
        _, _, mask = net.forward_ragged(T(d['mic']), T(d['far']), [m['n']], want_spec=False, want_mask=True)
    torch.cuda.synchronize()
    if m['version'] == 1:
        out_wav, out_spec, near_spec, loss = res
        assert abs(float(loss) - float(d['loss'])) <= 1e-4 * abs(float(d['loss']))
    else:
        out_spec, out_wav, near_spec = res
    out_wav, out_spec, near_spec = (x[0].cpu().numpy() for x in (out_wav, out_spec, near_spec))
    assert out_wav.shape == d['out_wav'].shape == (256 * (m['n'] // 256),)     # bit-exact framing
    assert out_spec.shape == d['out_spec'].shape == (514, m['n'] // 256 + 1)
    assert rel(out_wav, d['out_wav']) <= F32_TOL
    assert rel(out_spec, d['out_spec']) <= F32_TOL
    assert rel(near_spec, d['near_spec']) <= F32_TOL
    assert rel(mask[0].cpu().numpy(), d['mask']) <= F32_TOL


@pytest.mark.parametrize('name', ['v2E_2125', 'v1_2125', 'v2E_16000'])
def test_bf16_close_to_reference(name):
    net, m, _ = build(name, 'bf16')
    d = np.load(os.path.join(GOLD, f'crn_{name}.npz'))
    with torch.no_grad():
        out, _, mask = net.forward_ragged(T(d['mic']), T(d['far']), [m['n']], want_spec=False, want_mask=True)
    torch.cuda.synchronize()
    out = out[0].cpu().numpy()
    assert out.shape == d['out_wav'].shape
    assert np.isfinite(out).all()
    margin(f'bf16 {name} out_wav vs reference', rel(out, d['out_wav']), BF16_WAV_TOL)
    margin(f'bf16 {name} mask vs reference', rel(mask[0].cpu().numpy(), d['mask']), BF16_MASK_TOL)


@pytest.mark.parametrize('name', ['v2E_2125', 'v1_2125', 'v2E_16000'])
def test_fp8_close_to_reference(name):
    d = np.load(os.path.join(GOLD, f'crn_{name}.npz'))
    outs = {}
    for dt in ('bf16', 'fp8'):
        net, m, _ = build(name, dt)
        with torch.no_grad():
            out, _, mask = net.forward_ragged(T(d['mic']), T(d['far']), [m['n']], want_spec=False, want_mask=True)
        torch.cuda.synchronize()
        outs[dt] = (out[0].cpu().numpy(), mask[0].cpu().numpy())
    out, mask = outs['fp8']
    assert out.shape == d['out_wav'].shape
    assert np.isfinite(out).all()
    margin(f'fp8 {name} out_wav vs reference', rel(out, d['out_wav']), FP8_WAV_TOL)
    margin(f'fp8 {name} mask vs reference', rel(mask, d['mask']), FP8_MASK_TOL)
    margin(f'fp8 {name} out_wav vs bf16', rel(out, outs['bf16'][0]), FP8_VS_BF16_TOL)
    assert not np.array_equal(out, outs['bf16'][0])       # the MX path really ran


@pytest.mark.parametrize('dtype', ['f32', 'bf16', 'fp8'])
def test_ragged_batch_equals_single_calls(dtype):
    net, m, conf = build('v2E_2125', dtype)
    from aec_amd import synth
    lens = [3000, 1234, 4100, 256]
    sig = [synth.scene(n, 40 + i, return_echo=True) for i, n in enumerate(lens)]
    L = max(lens)
    pad = lambda k: torch.tensor(np.stack([np.pad(s[k], (0, L - len(s[k]))) for s in sig]), device='cuda:0')
    with torch.no_grad():
        bout, bspec, _ = net.forward_ragged(pad(0), pad(1), lens)
        singles = [net.forward_ragged(T(s[0]), T(s[1]), [len(s[0])]) for s in sig]
    torch.cuda.synchronize()
    for i, n in enumerate(lens):
        o1, s1, _ = singles[i]
        nout = 256 * (n // 256)
        tn = n // 256 + 1
        assert torch.equal(bout[i, :nout], o1[0]), i
        assert torch.equal(bspec[i, :, :tn], s1[0]), i
        assert not bout[i, nout:].any()


def test_f32_long_utterance_against_oracle():
    # 4 s utterance, full net_conf: the GPU recurrence over 251 frames vs the float64 oracle
    net, m, conf = build('v2E_2125', 'f32')
    from aec_amd import synth
    n = 64000
    mic, far, near, echo = synth.scene(n, 77, return_echo=True)
    with torch.no_grad():
        out, spec, _ = net.forward_ragged(T(mic), T(far), [n])
    torch.cuda.synchronize()
    w = C.make_weights(conf, 2, m['weight_seed'])
    r = C.forward(w, conf, 2, mic, far)
    assert out.shape[1] == r['out_wav'].shape[0]
    assert rel(out[0].cpu().numpy(), r['out_wav']) <= F32_TOL
    assert rel(spec[0].cpu().numpy(), r['out_spec']) <= F32_TOL


@pytest.mark.parametrize('graph', [False, True], ids=['direct', 'graph'])
@pytest.mark.parametrize('dtype', ['f32', 'bf16', 'fp8'])
def test_streaming_equals_batch(dtype, graph):
    """aec_crn_stream_step (the per-frame loop; its launches direct or
    replayed from the per-parity hipGraphs, whose input / output nodes are
    re-pointed at each call's buffers) reproduces the batch forward hop by
    hop, with per-stream reset mid-run.  The GEMMs, LSTM
    step and combine are the same kernels; the streaming front / back kernels
    restate the batch transforms, and the compiler contracts a few of their
    multiply-adds differently, so f32 agrees to ~1e-6 relative (observed max
    abs 2e-8 on 0.015-RMS output), not bit for bit.  Tolerance: relative RMS
    <= 1e-5 (f32), <= 1e-2 (bf16: a flipped bf16 rounding of an activation
    propagates)."""
    net, m, conf = build('v2E_2125', dtype)
    from aec_amd import synth
    lens = [2125, 1000, 2304]
    sig = [synth.scene(n, 60 + i, return_echo=True) for i, n in enumerate(lens)]
    B = len(lens)
    L = max(lens)
    pad = lambda k: torch.tensor(np.stack([np.pad(s[k], (0, L - len(s[k]))) for s in sig]), device='cuda:0')
    with torch.no_grad():
        ref_out, _, _ = net.forward_ragged(pad(0), pad(1), lens, want_spec=False)
    torch.cuda.synchronize()
    nh = L // 256 + 1                                   # hops fed per stream (last one zero-padded)
    mic = torch.zeros(B, 256 * (nh + 1), device='cuda:0')
    far = torch.zeros_like(mic)
    mic[:, :L] = pad(0)
    far[:, :L] = pad(1)
    net.stream_open(B, graph=graph)
    outs = []
    with torch.no_grad():
        for k in range(nh):
            outs.append(net.stream_step(mic[:, 256 * k:256 * (k + 1)], far[:, 256 * k:256 * (k + 1)]).clone())
    torch.cuda.synchronize()
    assert net.stream_stats() == dict(graph_mode=int(graph), graph_replays=nh if graph else 0,
                                      direct_hops=0 if graph else nh)
    got = torch.cat(outs[1:], dim=1)                    # step k emits hop k-1
    tol = {'f32': 1e-5, 'bf16': 1e-2, 'fp8': 2e-2}[dtype]
    for b, n in enumerate(lens):
        no = 256 * (n // 256)
        assert rel(got[b, :no].cpu(), ref_out[b, :no].cpu()) <= tol, (dtype, b)
    # reset stream 1 and run utterance 0 through it again: same output as batch row 0
    net.stream_reset(1)
    outs = []
    with torch.no_grad():
        for k in range(nh):
            mh = mic[:, 256 * k:256 * (k + 1)].clone()
            fh = far[:, 256 * k:256 * (k + 1)].clone()
            mh[1], fh[1] = mic[0, 256 * k:256 * (k + 1)], far[0, 256 * k:256 * (k + 1)]
            outs.append(net.stream_step(mh, fh)[1].clone())
    torch.cuda.synchronize()
    got1 = torch.cat(outs[1:])
    no = 256 * (lens[0] // 256)
    assert rel(got1[:no].cpu(), ref_out[0, :no].cpu()) <= tol


def test_bf16_batch256_embeds_goldens():
    """BASELINE config 3's shape: bf16, 256 rows in one call.  The reference
    golden utterances (full net_conf, v2 'E') sit in a 256-row ragged batch;
    they match the reference within the bf16 tolerance, and EVERY row equals
    its own single-utterance call bit for bit (no coupling across rows)."""
    net, m, conf = build('v2E_16000', 'bf16')
    from aec_amd import synth
    gold = {5: 'v2E_16000', 200: 'v2E_2125', 77: 'v2E_255'}
    for g in gold.values():
        assert META[g]['version'] == 2 and META[g]['overrides'] == {} and META[g]['weight_seed'] == m['weight_seed']
    rng = np.random.default_rng(256)
    B = 256
    rows = []
    for b in range(B):
        if b in gold:
            d = np.load(os.path.join(GOLD, f'crn_{gold[b]}.npz'))
            rows.append((d['mic'], d['far']))
        else:
            n = int(rng.integers(256, 4000))
            mic, far, _ = synth.scene(n, 3000 + b)
            rows.append((mic, far))
    lens = [len(r[0]) for r in rows]
    L = max(lens)
    pad = lambda k: torch.tensor(np.stack([np.pad(r[k], (0, L - len(r[k]))) for r in rows]), device='cuda:0')
    with torch.no_grad():
        bout, _, bmask = net.forward_ragged(pad(0), pad(1), lens, want_spec=False, want_mask=True)
    torch.cuda.synchronize()
    for b, g in gold.items():
        d = np.load(os.path.join(GOLD, f'crn_{g}.npz'))
        no = META[g]['out_len']
        o = bout[b, :no].cpu().numpy()
        assert o.shape == d['out_wav'].shape and np.isfinite(o).all()
        assert not bout[b, no:].any()
        if no:
            margin(f'bf16 ragged {g} out_wav vs reference', rel(o, d['out_wav']), BF16_WAV_TOL)
            tn = META[g]['n'] // 256 + 1
            margin(f'bf16 ragged {g} mask vs reference', rel(bmask[b][..., :tn].cpu().numpy(), d['mask']),
                   BF16_MASK_TOL)
    with torch.no_grad():
        for b in range(B):
            o1, _, _ = net.forward_ragged(T(rows[b][0]), T(rows[b][1]), [lens[b]], want_spec=False)
            no = 256 * (lens[b] // 256)
            assert torch.equal(bout[b, :no], o1[0, :no]), b
    torch.cuda.synchronize()


def test_persistent_recurrence_matches_step_kernel(monkeypatch):
    """The persistent LSTM recurrence (crn_persist.hip: one launch per layer,
    W_hh resident, h exchanged between the blocks of a team, two row halves
    in alternating phases) against
    the per-frame step kernel (AEC_CRN_PERSIST=0) on a 300-stream bf16 batch
    (two persistent launches per layer: 256 + 44 streams).  All are bf16 with
    f32 accumulation; the persistent kernels sum the two K halves separately
    (and use their own sigmoid / tanh algebra), so the bound is the
    bf16 one (relative RMS <= 1e-2), not bit equality.  A second call checks
    that the first left no timeout flag behind."""
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    from aec_amd import synth
    B, n = 300, 8000
    mic, far, _ = synth.batch(B, n, seed0=900)
    M, F = (torch.from_numpy(a).to('cuda:0') for a in (mic, far))
    outs = {}
    for flag in ('0', '1'):
        monkeypatch.setenv('AEC_CRN_PERSIST', flag)            # read when the handle is created
        net, m, conf = build('v2E_16000', 'bf16')
        with torch.no_grad():
            o, _, _ = net.forward_ragged(M, F, [n] * B, want_spec=False)
            o2, _, _ = net.forward_ragged(M[:3], F[:3], [n] * 3, want_spec=False)
        torch.cuda.synchronize()
        outs[flag] = (o.cpu().numpy(), o2.cpu().numpy())
    assert np.isfinite(outs['1'][0]).all()
    margin('persistent vs step kernel (bf16)', rel(outs['1'][0], outs['0'][0]), PERSIST_TOL)
    assert np.array_equal(outs['1'][1], outs['1'][0][:3])   # batch composition stays bit-exact


def test_persistent_timeout_fails_that_call(monkeypatch):
    """A persistent-grid timeout is reported by the call that hit it: with the
    poll targets made unreachable (AEC_CRN_PERSIST_STALL, read per call: a
    team that never arrives) and the poll bound cut to 64 polls
    (AEC_CRN_SPIN_LIMIT), every wave gives up waiting, the grid drains, and
    that forward_ragged raises; the next call with the normal settings on the
    same handle succeeds and equals a fresh handle's output bit for bit."""
    monkeypatch.delenv('AEC_CRN_PERSIST', raising=False)
    net, m, conf = build('v2E_16000', 'bf16')
    from aec_amd import synth
    B, n = 64, 32000
    mic, far, _ = synth.batch(B, n, seed0=950)
    M, F = (torch.from_numpy(a).to('cuda:0') for a in (mic, far))
    monkeypatch.setenv('AEC_CRN_SPIN_LIMIT', '64')
    monkeypatch.setenv('AEC_CRN_PERSIST_STALL', '1')
    with torch.no_grad(), pytest.raises(RuntimeError, match='timed out'):
        net.forward_ragged(M, F, [n] * B, want_spec=False)
    monkeypatch.delenv('AEC_CRN_SPIN_LIMIT')
    monkeypatch.delenv('AEC_CRN_PERSIST_STALL')
    with torch.no_grad():
        o, _, _ = net.forward_ragged(M, F, [n] * B, want_spec=False)
        fresh, _, _ = build('v2E_16000', 'bf16')
        o2, _, _ = fresh.forward_ragged(M, F, [n] * B, want_spec=False)
    torch.cuda.synchronize()
    assert torch.isfinite(o).all()
    assert torch.equal(o, o2)


@pytest.mark.parametrize('dtype', ['bf16', 'fp8'])
def test_c3_shape_long_rows_match_reference_port(dtype):
    """BASELINE config 3's exact shape: 256 streams x 160,000 samples in one
    call (626-frame bf16 / fp8 recurrence, the persistent LSTM kernel, the
    row GEMMs at their benchmark sizes).  Three far-end single-talk rows
    (first, middle, last) are checked against the reference op mix
    (oracle/torch_crn_port.py: conv2d / conv_transpose2d / nn.LSTM in f32,
    pinned to the reference goldens by tests/test_crn_oracle.py): out_wav
    relative RMS within the dtype's bar and ERLE within C3_ERLE_DB dB.  The
    other 253 rows are seeded noise scenes (they only have to be there)."""
    import sys
    net, m, conf = build('v2E_16000', dtype)
    from aec_amd import synth
    from torch_crn_port import TorchCrnPort
    import aec_oracle as O
    B, n = 256, 160000
    rows = (0, 131, 255)
    g = torch.Generator(device='cuda:0').manual_seed(31)
    M = 0.05 * torch.randn(B, n, device='cuda:0', generator=g)
    F = 0.1 * torch.randn(B, n, device='cuda:0', generator=g)
    sc = {r: synth.scene(n, 7100 + r, double_talk=False) for r in rows}
    for r in rows:
        M[r] = torch.from_numpy(sc[r][0]).cuda()
        F[r] = torch.from_numpy(sc[r][1]).cuda()
    with torch.no_grad():
        out, _, _ = net.forward_ragged(M, F, [n] * B, want_spec=False)
    torch.cuda.synchronize()
    got = out[list(rows)].cpu().numpy()
    assert got.shape == (3, 256 * (n // 256))
    assert np.isfinite(got).all()
    w = C.make_weights(conf, 2, m['weight_seed'])
    port = TorchCrnPort(w, conf, 2)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref = port(torch.from_numpy(np.stack([sc[r][0] for r in rows])),
               torch.from_numpy(np.stack([sc[r][1] for r in rows]))).numpy()
    tol = BF16_WAV_TOL if dtype == 'bf16' else FP8_WAV_TOL
    errs = [rel(got[i], ref[i]) for i in range(3)]
    d_erle = [O.erle_db(sc[r][0], got[i]) - O.erle_db(sc[r][0], ref[i]) for i, r in enumerate(rows)]
    margin(f'{dtype} C3 256x160000 rows vs reference op mix', max(errs), tol)
    margin(f'{dtype} C3 256x160000 |ERLE delta| dB', max(abs(d) for d in d_erle), C3_ERLE_DB)


def test_fp8_shadow_operands_bit_exact(monkeypatch):
    """dtype fp8: the MX-fp8 GEMMs read their e4m3 operands in place from
    shadows their producers' epilogues write (encoder / decoder GEMMs and the
    LSTM combine), with no quantisation pass; AEC_CRN_MX8_SHADOW=0 quantises
    the implicit rows first.  Same rule (E8M0 per 32 k from the bf16 values)
    on the same values, so the batch forward (ragged rows: M tails, conv
    padding taps) and the per-hop step are bit-identical."""
    from aec_amd import synth
    lens = [16000, 9000, 12345, 256, 4000]
    L = max(lens)
    sig = [synth.scene(n, 500 + i) for i, n in enumerate(lens)]
    pad = lambda k: torch.tensor(np.stack([np.pad(s[k], (0, L - len(s[k]))) for s in sig]), device='cuda:0')
    res = {}
    for flag in ('0', '1'):
        monkeypatch.setenv('AEC_CRN_MX8_SHADOW', flag)            # read when the handle is created
        net, m, conf = build('v2E_16000', 'fp8')
        with torch.no_grad():
            out, spec, _ = net.forward_ragged(pad(0), pad(1), lens)
            net.stream_open(len(lens))
            hops = [net.stream_step(pad(0)[:, 256 * k:256 * (k + 1)].contiguous(),
                                    pad(1)[:, 256 * k:256 * (k + 1)].contiguous()).clone() for k in range(12)]
        torch.cuda.synchronize()
        res[flag] = (out.cpu(), spec.cpu(), torch.stack(hops).cpu())
    (o0, s0, h0), (o1, s1, h1) = res['0'], res['1']
    assert torch.equal(o0, o1)
    assert torch.equal(h0, h1)
    for i, n in enumerate(lens):                        # frames past a row's end are unspecified
        tn = n // 256 + 1
        assert torch.equal(s0[i, :, :tn], s1[i, :, :tn]), i


def test_fp8_stream_mx_recurrence(monkeypatch):
    """dtype fp8 per-hop step (BASELINE config 5): the LSTM recurrence on the
    scaled MFMA (W_hh and h_{t-1} as e4m3 with an E8M0 scale per 32 k) with the
    NavieComplexLSTM combination fused into its epilogue (lstm_step_mx8_kernel)
    against the bf16 step + combine kernels (AEC_CRN_STEP_MX=0, read at
    stream_open) on 80 streams (three step blocks, the last one partial) of
    the full net_conf: within MX_VS_BF16_STEP_TOL relative RMS of each other per
    stream (observed 0.003-0.005: the e4m3 rounding of W_hh and h against
    bf16), and not identical (the MX recurrence really ran); three streams
    within the fp8 bar of the reference op mix (oracle/torch_crn_port), the
    parity gate proper."""
    from aec_amd import synth
    import torch_crn_port as P
    net, m, conf = build('v2E_16000', 'fp8')
    B, n = 80, 8000
    sig = [synth.scene(n, 1700 + b) for b in range(B)]
    nh = n // 256 + 1
    M = torch.zeros(B, 256 * (nh + 1), device='cuda:0')
    F = torch.zeros_like(M)
    M[:, :n] = torch.from_numpy(np.stack([s[0] for s in sig])).cuda()
    F[:, :n] = torch.from_numpy(np.stack([s[1] for s in sig])).cuda()
    res = {}
    for flag in ('0', '1'):
        monkeypatch.setenv('AEC_CRN_STEP_MX', flag)
        net.stream_open(B)
        with torch.no_grad():
            outs = [net.stream_step(M[:, 256 * k:256 * (k + 1)], F[:, 256 * k:256 * (k + 1)]).clone()
                    for k in range(nh)]
        torch.cuda.synchronize()
        res[flag] = torch.cat(outs[1:], dim=1)[:, :256 * (n // 256)].cpu().numpy()
    assert np.isfinite(res['1']).all()
    errs = [rel(res['1'][b], res['0'][b]) for b in range(B)]
    margin('fp8 stream MX vs bf16 recurrence (80 streams)', max(errs), MX_VS_BF16_STEP_TOL)
    assert not np.array_equal(res['1'], res['0'])
    w = C.make_weights(conf, 2, m['weight_seed'])
    port = P.TorchCrnPort(w, conf, 2)
    for b in (0, 40, 79):
        ref = port(torch.from_numpy(sig[b][0])[None], torch.from_numpy(sig[b][1])[None])[0].numpy()
        margin(f'fp8 stream MX stream {b} vs reference op mix', rel(res['1'][b], ref), FP8_WAV_TOL)


def test_fp8_stream_mx_scale_paths_bit_exact(monkeypatch):
    """The MX layer step's two scale paths (lstm_step_mx8_kernel): the K scales
    read per stage from LDS (AEC_CRN_MX_SREG=0, two stage buffers) and held in
    registers after a transposed pass through the third stage buffer (default
    at H = 1024) feed the same scale bytes to the same MFMAs, so 40 streams
    (two step blocks, the last one partial) of the full net_conf agree bit for
    bit over 12 hops."""
    from aec_amd import synth
    net, m, conf = build('v2E_16000', 'fp8')
    B, n = 40, 3072
    sig = [synth.scene(n, 2100 + b) for b in range(B)]
    nh = n // 256 + 1
    M = torch.zeros(B, 256 * (nh + 1), device='cuda:0')
    F = torch.zeros_like(M)
    M[:, :n] = torch.from_numpy(np.stack([s[0] for s in sig])).cuda()
    F[:, :n] = torch.from_numpy(np.stack([s[1] for s in sig])).cuda()
    monkeypatch.setenv('AEC_CRN_STEP_MX', '1')
    res = {}
    for flag in ('0', '1'):
        monkeypatch.setenv('AEC_CRN_MX_SREG', flag)
        net.stream_open(B)
        with torch.no_grad():
            outs = [net.stream_step(M[:, 256 * k:256 * (k + 1)], F[:, 256 * k:256 * (k + 1)]).clone()
                    for k in range(nh)]
        torch.cuda.synchronize()
        res[flag] = torch.cat(outs, dim=1).cpu().numpy()
    assert np.isfinite(res['1']).all()
    assert np.array_equal(res['1'], res['0'])


@pytest.mark.parametrize('name,dtype,nlms', [('v2E_16000', 'bf16', False), ('v2E_16000', 'fp8', False),
                                             ('v2E_16000', 'bf16', True), ('v2E_16000', 'fp8', True),
                                             ('v1_2125', 'bf16', True), ('v2C_bn_2125', 'fp8', False),
                                             ('v2R_1000', 'bf16', False)])
def test_fused_stream_bit_exact(monkeypatch, name, dtype, nlms):
    """The per-hop step's fused kernels (crn_stream.hip) against the separate
    launches (AEC_CRN_STREAM_FUSE=0, read at stream_open):
    * front: frame -> rFFT -> FD-NLMS step -> X0 -> encoder levels 0-2 in one
      launch (vs the front kernel, the NLMS kernel and three row GEMMs), with
      bit 2 level 3 as well (16 x 128, its MX-fp8 shadow written in the
      kernel for the fp8 level 4 that reads it);
    * back: decoder levels 3-1 with their skips, the mask (E / C / R), irFFT
      and overlap-add in one launch (vs three row GEMMs and the back kernel);
      with bit 3 (fp8) decoder level 4's MX-fp8 GEMM as well (scaled MFMA on
      cat[4]'s shadow, its split-K sum restated), and with bit 4 encoder
      level 4's in the front (on level 3's shadow kept in LDS): bit-identical
      to bits 3 and 4 off.
    The same transform code, NLMS arithmetic, 32-k MFMA chunks in the same
    order and epilogues: with the fused front alone (AEC_CRN_STREAM_FUSE=1,
    5) 37 streams over 14 hops agree bit for bit; with the fused back as well the
    masked spectrum reaches the inverse transform through LDS (the separate
    back kernel keeps its chain group's bins in registers, where the compiler
    contracts the mask's last product into the inverse pack), so the output
    moves by ~1 ulp (observed 54 of 18,944 samples, relative RMS 8e-10):
    bound 1e-6 relative RMS.  DCCRN v1 (tanh mask level) and v2 in every
    masking mode."""
    from aec_amd import synth
    m = META[name]
    conf = copy.deepcopy(aec_amd.net_conf)
    conf.update(m['overrides'])
    nl = dict(taps=4, mu=0.3, beta=0.5, delta=1e-4) if nlms else None
    net = (aec_amd.dccrn if m['version'] == 1 else aec_amd.dccrn2).DCCRN(conf, dtype=dtype, nlms=nl).eval()
    sd = net.state_dict()
    for k, v in C.make_weights(conf, m['version'], m['weight_seed']).items():
        sd[k] = torch.from_numpy(v)
    net.load_state_dict(sd, strict=True)
    net = net.to('cuda:0')
    B, n = 37, 3328
    sig = [synth.scene(n, 2900 + b) for b in range(B)]
    nh = n // 256 + 1
    M = torch.zeros(B, 256 * (nh + 1), device='cuda:0')
    F = torch.zeros_like(M)
    M[:, :n] = torch.from_numpy(np.stack([s[0] for s in sig])).cuda()
    F[:, :n] = torch.from_numpy(np.stack([s[1] for s in sig])).cuda()
    res = {}
    for flag in ('0', '1', '5', '3', '7', '15', '31'):
        monkeypatch.setenv('AEC_CRN_STREAM_FUSE', flag)
        net.stream_open(B)
        with torch.no_grad():
            outs = [net.stream_step(M[:, 256 * k:256 * (k + 1)], F[:, 256 * k:256 * (k + 1)]).clone()
                    for k in range(nh)]
        torch.cuda.synchronize()
        res[flag] = torch.cat(outs, dim=1).cpu().numpy()
    assert np.isfinite(res['3']).all()
    assert np.abs(res['3']).max() > 0
    assert np.array_equal(res['1'], res['0'])
    assert np.array_equal(res['5'], res['0'])
    assert rel(res['3'], res['0']) <= 1e-6
    assert rel(res['7'], res['0']) <= 1e-6
    assert np.array_equal(res['15'], res['7'])
    assert np.array_equal(res['31'], res['7'])


@pytest.mark.parametrize('dtype', ['bf16', 'fp8'])
def test_lstm_combine_vector_form_bit_exact(monkeypatch, dtype):
    """NavieComplexLSTM's real / imag combination (dccrn.py:443-446) in its 8-units-per-thread form
    (16-B row loads and stores, the MX shadow's 32-unit group over 4 lanes) against the one-unit
    form (CRN_COMBINE_VEC=0, read per call): the same per-element bf16 arithmetic and E8M0 rule, so
    the batch forward's output is bit-identical (5 ragged streams of net_conf)."""
    from aec_amd import synth
    net, m, conf = build('v2E_16000', dtype)
    lens = [16000, 12345, 9000, 16000, 4100]
    sig = [synth.scene(n, 4200 + b) for b, n in enumerate(lens)]
    mic = torch.zeros(len(lens), max(lens), device='cuda:0')
    far = torch.zeros_like(mic)
    for b, sc in enumerate(sig):
        mic[b, :lens[b]] = torch.from_numpy(sc[0])
        far[b, :lens[b]] = torch.from_numpy(sc[1])
    res = {}
    for flag in ('0', '1'):
        monkeypatch.setenv('CRN_COMBINE_VEC', flag)
        with torch.no_grad():
            out, _, _ = net.forward_ragged(mic, far, lens, want_spec=False)
        torch.cuda.synchronize()
        res[flag] = out.cpu().numpy()
    assert np.isfinite(res['1']).all() and np.abs(res['1']).max() > 0
    assert np.array_equal(res['1'], res['0'])


def test_fp8_stream_fold_policy_bit_exact():
    """The per-hop step folds the MX-fp8 encoder level 4 / decoder level cl = 4 into the fused front
    / back only while every stream has a CU of its own (aec_crn_stream_open: streams <= CUs; past
    that the unfolded kernels' occupancy wins, profiles/r04v_c5_fold_sweep.txt).  Both forms run
    the same MFMA chains and epilogues and every stream's rows are independent of the others, so
    37 streams (folds on) and the same 37 streams inside a CUs + 44 stream handle (folds off) agree
    bit for bit over 13 hops: net_conf, fp8, 4-tap FD-NLMS (BASELINE config 5's step)."""
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    from aec_amd import synth
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    m = META['v2E_16000']
    conf = copy.deepcopy(aec_amd.net_conf)
    conf.update(m['overrides'])
    net = aec_amd.dccrn2.DCCRN(conf, dtype='fp8', nlms=dict(taps=4, mu=0.3, beta=0.5, delta=1e-4)).eval()
    sd = net.state_dict()
    for k, v in C.make_weights(conf, 2, m['weight_seed']).items():
        sd[k] = torch.from_numpy(v)
    net.load_state_dict(sd, strict=True)
    net = net.to('cuda:0')
    n, Bs, Bb = 3072, 37, ncu + 44
    nh = n // 256 + 1
    sig = [synth.scene(n, 3100 + b) for b in range(Bs)]
    M = torch.zeros(Bb, 256 * (nh + 1), device='cuda:0')
    F = torch.zeros_like(M)
    M[:Bs, :n] = torch.from_numpy(np.stack([s[0] for s in sig])).cuda()
    F[:Bs, :n] = torch.from_numpy(np.stack([s[1] for s in sig])).cuda()
    g = torch.Generator(device='cuda:0').manual_seed(7)
    M[Bs:, :n] = 0.1 * torch.randn(Bb - Bs, n, device='cuda:0', generator=g)
    F[Bs:, :n] = 0.1 * torch.randn(Bb - Bs, n, device='cuda:0', generator=g)
    res = {}
    for B in (Bs, Bb):
        net.stream_open(B)
        with torch.no_grad():
            outs = [net.stream_step(M[:B, 256 * k:256 * (k + 1)], F[:B, 256 * k:256 * (k + 1)]).clone()
                    for k in range(nh)]
        torch.cuda.synchronize()
        res[B] = torch.cat(outs, dim=1).cpu().numpy()
    assert np.isfinite(res[Bb]).all()
    assert np.abs(res[Bs]).max() > 0
    assert np.array_equal(res[Bb][:Bs], res[Bs])


@pytest.mark.parametrize('name,dtype,nlms', [('v2E_16000', 'bf16', False), ('v2E_16000', 'fp8', True),
                                             ('v1_2125', 'bf16', True), ('v1_2125', 'bf16', False),
                                             ('v2C_bn_2125', 'fp8', False), ('v2R_1000', 'bf16', False)])
def test_back_mask_level_matches_gemm(monkeypatch, name, dtype, nlms):
    """Batch path, bf16 storage: the mask level (the last decoder level, 2
    output channels x 2 parities) computed inside the back kernel from cat[1]
    against the row GEMM writing the f32 mask to HBM (AEC_CRN_BACK_MASK=0, read
    per call): the same 32-k bf16 MFMA chunks from zero, the same bias / tanh
    epilogue, so out_wav and out_spec agree bit for bit.  Ragged lengths (dead
    frames of short rows are never computed) and the caller-wants-the-mask
    case (want_mask: the GEMM path, the mask equal to the fused run's)."""
    from aec_amd import synth
    m = META[name]
    conf = copy.deepcopy(aec_amd.net_conf)
    conf.update(m['overrides'])
    nl = dict(taps=4, mu=0.3, beta=0.5, delta=1e-4) if nlms else None
    net = (aec_amd.dccrn if m['version'] == 1 else aec_amd.dccrn2).DCCRN(conf, dtype=dtype, nlms=nl).eval()
    sd = net.state_dict()
    for k, v in C.make_weights(conf, m['version'], m['weight_seed']).items():
        sd[k] = torch.from_numpy(v)
    net.load_state_dict(sd, strict=True)
    net = net.to('cuda:0')
    B, n = 23, 9000
    lens = [n - 317 * b for b in range(B)]
    M = torch.zeros(B, n, device='cuda:0')
    F = torch.zeros_like(M)
    for b in range(B):
        s = synth.scene(lens[b], 3100 + b)
        M[b, :lens[b]] = torch.from_numpy(s[0]).cuda()
        F[b, :lens[b]] = torch.from_numpy(s[1]).cuda()
    res = {}
    for flag in ('0', '1'):
        monkeypatch.setenv('AEC_CRN_BACK_MASK', flag)
        with torch.no_grad():
            out, spec, _ = net.forward_ragged(M, F, lens, want_spec=True)
        torch.cuda.synchronize()
        res[flag] = (out.cpu().numpy(), spec.cpu().numpy())
    with torch.no_grad():
        out_m, _, mask = net.forward_ragged(M, F, lens, want_spec=False, want_mask=True)
    torch.cuda.synchronize()
    assert np.isfinite(res['1'][0]).all() and np.abs(res['1'][0]).max() > 0
    for b in range(B):
        nb, tb = 256 * (lens[b] // 256), lens[b] // 256 + 1
        assert np.array_equal(res['1'][0][b, :nb], res['0'][0][b, :nb]), b
        assert np.array_equal(res['1'][1][b, :, :tb], res['0'][1][b, :, :tb]), b
        assert np.array_equal(out_m.cpu().numpy()[b, :nb], res['1'][0][b, :nb]), b
    assert np.isfinite(mask.cpu().numpy()).all()


@pytest.mark.parametrize('knob', ['AEC_CRN_BATCH_ENC', 'AEC_CRN_BATCH_DEC'])
@pytest.mark.parametrize('name,dtype,nlms', [('v2E_16000', 'bf16', False), ('v2E_16000', 'fp8', False),
                                             ('v2E_16000', 'bf16', True), ('v1_2125', 'bf16', False),
                                             ('v2C_bn_2125', 'fp8', True)])
def test_batch_fused_levels_bit_exact(monkeypatch, knob, name, dtype, nlms):
    """Batch path, bf16 storage, the fused conv levels against the row GEMMs
    they replace (knob=0, read per call; knob=2 fails the call unless the
    fused kernel ran):
    * AEC_CRN_BATCH_ENC: encoder levels 0-3 in one persistent launch
      (crn_enc_batch_kernel: X0 -> the four maps in LDS, four frames per
      block, level 3's MX-fp8 shadow written in the kernel);
    * AEC_CRN_BATCH_DEC: decoder levels cl = 3, 2 in one persistent launch
      (crn_dec_batch_kernel: cat[3] -> cat[2]'s decoder half in LDS ->
      cat[1]'s decoder half).
    The same packed weights, 32-k bf16 MFMA chunks from zero and PReLU
    epilogue, so out_wav and out_spec agree bit for bit.  Ragged lengths;
    F = 23 rows x 36 frames is not a multiple of the block's four frames
    (the tail iteration)."""
    from aec_amd import synth
    m = META[name]
    conf = copy.deepcopy(aec_amd.net_conf)
    conf.update(m['overrides'])
    nl = dict(taps=4, mu=0.3, beta=0.5, delta=1e-4) if nlms else None
    net = (aec_amd.dccrn if m['version'] == 1 else aec_amd.dccrn2).DCCRN(conf, dtype=dtype, nlms=nl).eval()
    sd = net.state_dict()
    for k, v in C.make_weights(conf, m['version'], m['weight_seed']).items():
        sd[k] = torch.from_numpy(v)
    net.load_state_dict(sd, strict=True)
    net = net.to('cuda:0')
    B, n = 23, 9000
    lens = [n - 317 * b for b in range(B)]
    M = torch.zeros(B, n, device='cuda:0')
    F = torch.zeros_like(M)
    for b in range(B):
        s = synth.scene(lens[b], 3300 + b)
        M[b, :lens[b]] = torch.from_numpy(s[0]).cuda()
        F[b, :lens[b]] = torch.from_numpy(s[1]).cuda()
    res = {}
    for flag in ('0', '2'):
        monkeypatch.setenv(knob, flag)
        with torch.no_grad():
            out, spec, _ = net.forward_ragged(M, F, lens, want_spec=True)
        torch.cuda.synchronize()
        res[flag] = (out.cpu().numpy(), spec.cpu().numpy())
    assert np.isfinite(res['2'][0]).all() and np.abs(res['2'][0]).max() > 0
    for b in range(B):
        nb, tb = 256 * (lens[b] // 256), lens[b] // 256 + 1
        assert np.array_equal(res['2'][0][b, :nb], res['0'][0][b, :nb]), b
        assert np.array_equal(res['2'][1][b, :, :tb], res['0'][1][b, :, :tb]), b
