"""GPU parity of the NLMS -> CRN composition (include/aec_crn.h with
nlms_taps > 0; SURVEY.md §8 a13 + a14): the FD-NLMS error spectrum E replaces
the mic spectrum as the DCCRN's mic channels and as the spectrum its mask is
applied to.

The composition has no reference counterpart (the reference runs the CRN on
the raw mic spectrum), so the oracle is ``crn_oracle.forward(..., nlms=...)``:
the float64 CRN restatement pinned by the reference's goldens
(tests/test_crn_oracle.py) fed by ``aec_oracle.nlms`` (the published NLMS
recursion, pinned in tests/test_oracle_golden.py).  Tolerances (relative RMS,
written here):

* E (the NLMS error spectrum, fp32 recursion vs float64): <= 1e-4;
* f32 network fed E: out_wav, out_spec, mask <= 1e-4 (the CRN's own f32 bar);
  v1 loss within 1e-4 relative;
* bf16 network fed E: out_wav <= 1e-2 (the CRN's bf16 bar);
* fp8 per-hop step (64 streams): every stream within 2e-2 of the fp8 batch
  forward, three within the CRN's fp8 bar (2e-2) of the oracle;
* streaming (per-hop step, NLMS state carried per stream)
  vs batch: <= 1e-5 f32 (the CRN streaming bar; the NLMS arithmetic itself is
  the same NlmsBin code on the same fp32 operands);
* batch composition (ragged rows in one call vs one call per row): bit-exact.
"""
import copy
import json
import os

import numpy as np
import pytest
import torch

import aec_amd
import crn_oracle as C
from aec_amd import synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
META = json.load(open(os.path.join(GOLD, 'crn_meta.json')))
NLMS = dict(taps=4, mu=0.3, beta=0.5, delta=1e-4)
E_TOL = 1e-4
F32_TOL = 1e-4
BF16_WAV_TOL = 1e-2


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-30))


def build(name, dtype, nlms=NLMS):
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    m = META[name]
    conf = copy.deepcopy(aec_amd.net_conf)
    conf.update(m['overrides'])
    net = (aec_amd.dccrn if m['version'] == 1 else aec_amd.dccrn2).DCCRN(conf, dtype=dtype, nlms=nlms).eval()
    w = C.make_weights(conf, m['version'], m['weight_seed'])
    sd = net.state_dict()
    for k, v in w.items():
        sd[k] = torch.from_numpy(v)
    net.load_state_dict(sd, strict=True)
    return net.to('cuda:0'), m, conf, w


def T(a):
    return torch.as_tensor(np.asarray(a), device='cuda:0')[None]


@pytest.mark.parametrize('name', ['v1_2125', 'v2E_2125', 'v2C_bn_2125', 'v2R_1000'])
def test_f32_nlms_crn_matches_oracle(name):
    net, m, conf, w = build(name, 'f32')
    n = 16000
    mic, far, near, echo = synth.scene(n, 91, return_echo=True)
    with torch.no_grad():
        res = net(T(mic), T(far), T(near), T(echo))
        E = net.error_spectra('cuda:0')
        _, _, mask = net.forward_ragged(T(mic), T(far), [n], want_spec=False, want_mask=True)
    torch.cuda.synchronize()
    r = C.forward(w, conf, m['version'], mic, far, near, echo, nlms=NLMS)
    if m['version'] == 1:
        out_wav, out_spec, _, loss = res
        assert abs(float(loss) - r['loss']) <= 1e-4 * abs(r['loss'])
    else:
        out_spec, out_wav, _ = res
    assert rel(E[0].cpu().numpy(), r['err_spec']) <= E_TOL
    assert out_wav.shape[1] == r['out_wav'].shape[0] == 256 * (n // 256)
    assert rel(out_wav[0].cpu().numpy(), r['out_wav']) <= F32_TOL
    assert rel(out_spec[0].cpu().numpy(), r['out_spec']) <= F32_TOL
    assert rel(mask[0].cpu().numpy(), r['mask']) <= F32_TOL
    # the NLMS really ran: E differs from the mic spectrum, and so does the output of the plain network
    plain, _, _, _ = build(name, 'f32', nlms=None)
    with torch.no_grad():
        o0, _, _ = plain.forward_ragged(T(mic), T(far), [n], want_spec=False)
    assert rel(o0[0].cpu().numpy(), r['out_wav']) > 10 * F32_TOL


def test_bf16_nlms_crn_close_to_oracle():
    net, m, conf, w = build('v2E_2125', 'bf16')
    n = 16000
    mic, far, _, _ = synth.scene(n, 92, return_echo=True)
    with torch.no_grad():
        out, _, _ = net.forward_ragged(T(mic), T(far), [n], want_spec=False)
    torch.cuda.synchronize()
    r = C.forward(w, conf, 2, mic, far, nlms=NLMS)
    o = out[0].cpu().numpy()
    assert np.isfinite(o).all()
    assert rel(o, r['out_wav']) <= BF16_WAV_TOL


@pytest.mark.parametrize('dtype', ['f32', 'bf16'])
def test_nlms_ragged_batch_equals_single_calls(dtype):
    net, m, conf, _ = build('v2E_2125', dtype)
    lens = [3000, 1234, 4100, 256]
    sig = [synth.scene(n, 140 + i, return_echo=True) for i, n in enumerate(lens)]
    L = max(lens)
    pad = lambda k: torch.tensor(np.stack([np.pad(s[k], (0, L - len(s[k]))) for s in sig]), device='cuda:0')
    with torch.no_grad():
        bout, bspec, _ = net.forward_ragged(pad(0), pad(1), lens)
        bE = net.error_spectra('cuda:0')
        singles = []
        for s in sig:
            o1, s1, _ = net.forward_ragged(T(s[0]), T(s[1]), [len(s[0])])
            singles.append((o1, s1, net.error_spectra('cuda:0')))
    torch.cuda.synchronize()
    for i, n in enumerate(lens):
        o1, s1, e1 = singles[i]
        nout = 256 * (n // 256)
        tn = n // 256 + 1
        assert torch.equal(bout[i, :nout], o1[0]), i
        assert torch.equal(bspec[i, :, :tn], s1[0]), i
        assert torch.equal(bE[i, :, :tn], e1[0]), i
        assert not bE[i, :, tn:].any(), i
        assert not bout[i, nout:].any()


@pytest.mark.parametrize('taps', [1, 4, 8])
def test_nlms_stream_step_equals_batch_and_oracle(taps):
    """The per-hop NLMS -> CRN step (aec_crn_stream_step, direct launches) reproduces the batch forward and the oracle, with a per-stream
    reset (the NLMS state of that stream restarts) mid-run."""
    nl = dict(NLMS, taps=taps)
    net, m, conf, w = build('v2E_2125', 'f32', nlms=nl)
    lens = [2125, 1000, 2304]
    sig = [synth.scene(n, 160 + i, return_echo=True) for i, n in enumerate(lens)]
    B = len(lens)
    L = max(lens)
    pad = lambda k: torch.tensor(np.stack([np.pad(s[k], (0, L - len(s[k]))) for s in sig]), device='cuda:0')
    with torch.no_grad():
        ref_out, _, _ = net.forward_ragged(pad(0), pad(1), lens, want_spec=False)
    torch.cuda.synchronize()
    nh = L // 256 + 1
    mic = torch.zeros(B, 256 * (nh + 1), device='cuda:0')
    far = torch.zeros_like(mic)
    mic[:, :L] = pad(0)
    far[:, :L] = pad(1)
    net.stream_open(B)
    outs = []
    with torch.no_grad():
        for k in range(nh):
            outs.append(net.stream_step(mic[:, 256 * k:256 * (k + 1)], far[:, 256 * k:256 * (k + 1)]).clone())
    torch.cuda.synchronize()
    got = torch.cat(outs[1:], dim=1)
    for b, n in enumerate(lens):
        no = 256 * (n // 256)
        assert rel(got[b, :no].cpu(), ref_out[b, :no].cpu()) <= 1e-5, b
    r = C.forward(w, conf, 2, sig[0][0], sig[0][1], nlms=nl)
    assert rel(got[0, :256 * (lens[0] // 256)].cpu(), r['out_wav']) <= F32_TOL
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
    assert rel(got1[:no].cpu(), ref_out[0, :no].cpu()) <= 1e-5


def test_error_spec_needs_nlms_handle():
    net, _, _, _ = build('v2E_2125', 'f32', nlms=None)
    with pytest.raises(RuntimeError):
        net.error_spectra('cuda:0')


FP8_WAV_TOL = 2e-2


def test_fp8_nlms_stream_step_close_to_oracle():
    """BASELINE config 5's unit: the per-hop step (direct launches) with the
    FD-NLMS in front and MX-fp8 GEMMs (dtype 'fp8'), 64 concurrent streams
    (the 64 x 64-tile MX GEMM at M = 64 x 128 bins), against the fp8 batch
    forward of the same network for every stream (<= 2e-2: the step kernels
    are the batch kernels; the streaming front / back restate the batch
    transforms) and against the float64 oracle (crn_oracle + aec_oracle.nlms)
    for three streams within the fp8 bar of tests/test_gpu_crn.py."""
    net, m, conf, w = build('v2E_2125', 'fp8')
    B, n = 64, 16000
    sig = [synth.scene(n, 930 + b, return_echo=True) for b in range(B)]
    nh = n // 256 + 1
    M = torch.zeros(B, 256 * (nh + 1), device='cuda:0')
    F = torch.zeros_like(M)
    M[:, :n] = torch.from_numpy(np.stack([s[0] for s in sig])).cuda()
    F[:, :n] = torch.from_numpy(np.stack([s[1] for s in sig])).cuda()
    net.stream_open(B)
    outs = []
    with torch.no_grad():
        for k in range(nh):
            outs.append(net.stream_step(M[:, 256 * k:256 * (k + 1)], F[:, 256 * k:256 * (k + 1)]).clone())
        ref_out, _, _ = net.forward_ragged(M[:, :n].contiguous(), F[:, :n].contiguous(), [n] * B, want_spec=False)
    torch.cuda.synchronize()
    no = 256 * (n // 256)
    got = torch.cat(outs[1:], dim=1)[:, :no].cpu().numpy()
    ref_out = ref_out.cpu().numpy()
    assert np.isfinite(got).all()
    errs = [rel(got[b], ref_out[b]) for b in range(B)]
    assert max(errs) <= 2e-2, (int(np.argmax(errs)), max(errs))
    for b in (0, 31, 63):
        r = C.forward(w, conf, 2, sig[b][0], sig[b][1], nlms=NLMS)
        assert rel(got[b], r['out_wav']) <= FP8_WAV_TOL, b
