"""CPU: the DCCRN oracle (oracle/crn_oracle.py) against the golden vectors the
reference itself produced (tests/golden/make_crn_golden.py).

Pins the float64 restatement of dccrn.py / dccrn2.py
before the GPU parity tests trust it.  Tolerance: relative RMS <= 1e-5 on
every stored tensor (observed ~6e-7: float64 restatement vs the reference's
float32 CPU path); framing integers exact.
"""
import json
import os

import numpy as np
import pytest

import crn_oracle as C

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
META = json.load(open(os.path.join(GOLD, 'crn_meta.json')))


def rel(a, b):
    b = np.asarray(b, np.float64)
    if b.size == 0:
        return 0.0
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-30))


@pytest.mark.parametrize('name', sorted(META))
def test_oracle_matches_reference(name):
    m = META[name]
    d = np.load(os.path.join(GOLD, f'crn_{name}.npz'))
    conf = dict(C.NET_CONF)
    conf.update(m['overrides'])
    w = C.make_weights(conf, m['version'], m['weight_seed'])
    cap = {}
    r = C.forward(w, conf, m['version'], d['mic'], d['far'], d['near'], d['echo'], capture=cap)
    assert r['out_wav'].shape == d['out_wav'].shape == (256 * (m['n'] // 256),)
    assert r['out_spec'].shape == d['out_spec'].shape == (514, m['n'] // 256 + 1)
    assert rel(r['out_wav'], d['out_wav']) <= 1e-5
    assert rel(r['out_spec'], d['out_spec']) <= 1e-5
    assert rel(r['mask'], d['mask']) <= 1e-5
    assert rel(r['near_spec'], d['near_spec']) <= 1e-5
    if 'enc0' in d:
        assert rel(cap['enc'][0], d['enc0']) <= 1e-5
    if 'loss' in d:
        assert abs(r['loss'] - float(d['loss'])) <= 1e-5 * abs(float(d['loss']))


def test_param_shapes_cover_reference_names():
    # the fixture weights name exactly the parameters / eval buffers the
    # reference state_dict holds for these configs (make_crn_golden asserts the
    # load was complete); spot-check the published sizes
    n2 = sum(int(np.prod(s)) for k, s in C.param_shapes(C.NET_CONF, 2) if not k.split('.')[-1].startswith(('RM', 'RV')))
    n1 = sum(int(np.prod(s)) for k, s in C.param_shapes(C.NET_CONF, 1) if not k.split('.')[-1].startswith('running'))
    assert n2 == 34902237
    assert n1 == 34885105


@pytest.mark.parametrize('name', ['v2E_2125', 'v1_2125', 'v2C_bn_2125', 'v2R_1000'])
def test_torch_port_matches_reference(name):
    # the CPU baseline of bench.py --pipeline crn (reference op mix, float32)
    import torch
    from torch_crn_port import TorchCrnPort
    m = META[name]
    d = np.load(os.path.join(GOLD, f'crn_{name}.npz'))
    conf = dict(C.NET_CONF)
    conf.update(m['overrides'])
    port = TorchCrnPort(C.make_weights(conf, m['version'], m['weight_seed']), conf, m['version'])
    out = port(torch.from_numpy(d['mic'])[None], torch.from_numpy(d['far'])[None])[0].numpy()
    assert out.shape == d['out_wav'].shape
    assert rel(out, d['out_wav']) <= 1e-4


@pytest.mark.parametrize('name', ['v2E_2125', 'v1_2125'])
def test_torch_port_nlms_matches_oracle(name):
    # the NLMS -> CRN composition (no reference counterpart): the torch port's
    # NLMS front end (the checker of the C4 bench-shape GPU test) against the
    # float64 oracle's, on a 1 s far-end single-talk scene
    import torch
    from torch_crn_port import TorchCrnPort
    from aec_amd import synth
    nl = dict(taps=4, mu=0.3, beta=0.5, delta=1e-4)
    m = META[name]
    conf = dict(C.NET_CONF)
    conf.update(m['overrides'])
    w = C.make_weights(conf, m['version'], m['weight_seed'])
    mic, far, _ = synth.scene(16000, 321, double_talk=False)
    r = C.forward(w, conf, m['version'], mic, far, nlms=nl)
    port = TorchCrnPort(w, conf, m['version'], nlms=nl)
    out = port(torch.from_numpy(mic)[None], torch.from_numpy(far)[None])[0].numpy()
    assert rel(out, r['out_wav']) <= 1e-4
    plain = TorchCrnPort(w, conf, m['version'])(torch.from_numpy(mic)[None], torch.from_numpy(far)[None])[0].numpy()
    assert rel(plain, r['out_wav']) > 1e-2          # the NLMS really ran



@pytest.mark.parametrize('nlms', [None, dict(taps=4, mu=0.3, beta=0.5, delta=1e-4)])
def test_torch_stream_port_equals_batch_port(nlms):
    # bench.py's c5_stream_fp8 cpu_baseline: the port stepped one hop per call
    # reproduces the batch port (step s emits hop s-1 of out_wav)
    import torch
    from torch_crn_port import TorchCrnPort, TorchCrnStreamPort
    from aec_amd import synth
    m = META['v2E_2125']
    conf = dict(C.NET_CONF)
    w = C.make_weights(conf, 2, m['weight_seed'])
    n, B = 2560, 2
    sig = [synth.scene(n, 400 + b) for b in range(B)]
    mic = torch.from_numpy(np.stack([s[0] for s in sig]))
    far = torch.from_numpy(np.stack([s[1] for s in sig]))
    ref = TorchCrnPort(w, conf, 2, nlms=nlms)(mic, far).numpy()
    sp = TorchCrnStreamPort(w, conf, 2, nlms=nlms)
    sp.stream_open(B)
    nh = n // 256 + 1
    pad = lambda x: torch.nn.functional.pad(x, [0, 256 * nh - n])
    mic, far = pad(mic), pad(far)
    hops = [sp.step(mic[:, 256 * k:256 * (k + 1)], far[:, 256 * k:256 * (k + 1)]) for k in range(nh)]
    got = torch.cat(hops[1:], 1).numpy()[:, :ref.shape[1]]
    assert got.shape == ref.shape
    assert rel(got, ref) <= 1e-4
