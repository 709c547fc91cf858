"""CPU: the DCCRN boundary — C-ABI exports (include/aec_crn.h), parameter
blob layout, state_dict compatibility with the reference names and the
no-CPU-fallback rule.  No GPU needed."""
import copy
import os
import re

import numpy as np
import pytest
import torch

import aec_amd
import crn_oracle as C
from aec_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_clib_exports_every_crn_symbol():
    hdr = open(os.path.join(REPO, 'include', 'aec_crn.h')).read()
    declared = set(re.findall(r'^\s*(?:[A-Za-z_][\w\s\*]*?)\b(aec_crn_\w+)\s*\(', hdr, re.M))
    assert declared == set(_lib.CRN_EXPORTS), declared ^ set(_lib.CRN_EXPORTS)
    lib = _lib.load()
    for s in declared:
        assert hasattr(lib, s), s


@pytest.mark.parametrize('version,over', [(1, {}), (2, {}), (2, {'use_cbn': False, 'masking_mode': 'C'}),
                                          (2, {'masking_mode': 'R', 'rnn_layers': 1})])
def test_param_blob_layout(version, over):
    conf = copy.deepcopy(aec_amd.net_conf)
    conf.update(over)
    net = (aec_amd.dccrn if version == 1 else aec_amd.dccrn2).DCCRN(conf)
    names = net.param_names()
    # same names and order as the oracle's restatement of the reference state_dict
    assert names == [n for n, _ in C.param_shapes(conf, version)]
    sd = net.state_dict()
    assert _lib.crn_param_count(version, conf) == sum(sd[n].numel() for n in names)
    blob = net.params_blob()
    assert blob.dtype == np.float32 and blob.size == _lib.crn_param_count(version, conf)


def test_unsupported_configs_rejected():
    bad = copy.deepcopy(aec_amd.net_conf)
    bad['conv_channels'] = [4, 16, 32, 64, 128, 256]      # 256 >> 5 = 8 != 4
    assert _lib.crn_param_count(2, bad) == 0
    bad = copy.deepcopy(aec_amd.net_conf)
    bad['hidden_dim'] = 8
    assert _lib.crn_param_count(2, bad) == 0


def test_nlms_config_validated_and_laid_out():
    import ctypes
    # aec_crn_config: 16 int32 fields then nlms_taps / mu / beta / delta (include/aec_crn.h)
    assert ctypes.sizeof(_lib.CrnConfig) == 20 * 4
    assert _lib.CrnConfig.nlms_taps.offset == 16 * 4
    lib = _lib.load()
    conf = aec_amd.net_conf
    good = _lib.crn_config(2, conf, 'f32', dict(taps=4, mu=0.3, beta=0.5, delta=1e-4))
    assert lib.aec_crn_param_count(ctypes.byref(good)) == _lib.crn_param_count(2, conf)   # same blob
    for bad in (dict(taps=9), dict(taps=4, mu=2.0), dict(taps=4, beta=1.0), dict(taps=4, delta=0.0)):
        c = _lib.crn_config(2, conf, 'f32', dict(dict(taps=4, mu=0.3, beta=0.5, delta=1e-4), **bad))
        assert lib.aec_crn_param_count(ctypes.byref(c)) == 0, bad


def test_oracle_nlms_front_end():
    """crn_oracle.forward(nlms=...) replaces the mic spectrum by aec_oracle.nlms's
    error: mu = 0 leaves E = X_mic (the plain network, bit for bit), and E is
    exactly the recursion applied to the two ConvSTFT spectra."""
    import aec_oracle as A
    from aec_amd import synth
    conf = copy.deepcopy(aec_amd.net_conf)
    conf['conv_channels'] = [4, 8, 8, 8, 8, 8, 8]
    w = C.make_weights(conf, 2, 3)
    mic, far, _ = synth.scene(3000, 5)
    plain = C.forward(w, conf, 2, mic, far)
    mu0 = C.forward(w, conf, 2, mic, far, nlms=dict(taps=4, mu=0.0, beta=0.5, delta=1e-4))
    assert np.array_equal(plain['out_wav'], mu0['out_wav'])
    r = C.forward(w, conf, 2, mic, far, nlms=dict(taps=2, mu=0.5, beta=0.9, delta=1e-3))
    E = A.nlms(A.stft(mic), A.stft(far), taps=2, mu=0.5, beta=0.9, delta=1e-3)
    assert np.array_equal(r['err_spec'], np.concatenate([E.real.T, E.imag.T], axis=0))
    assert not np.allclose(r['out_wav'], plain['out_wav'])


def test_fixture_weights_load_strictly_by_reference_names():
    for version, mod in ((1, aec_amd.dccrn), (2, aec_amd.dccrn2)):
        net = mod.DCCRN(aec_amd.net_conf)
        w = C.make_weights(aec_amd.net_conf, version, 7)
        sd = net.state_dict()
        for k, v in w.items():
            assert tuple(sd[k].shape) == v.shape, k
            sd[k] = torch.from_numpy(v)
        net.load_state_dict(sd, strict=True)
        blob = net.params_blob()
        exp = np.concatenate([w[n].reshape(-1) for n in net.param_names()])
        assert np.array_equal(blob, exp)


def test_crn_cpu_tensors_fail_loudly():
    net = aec_amd.dccrn2.DCCRN(aec_amd.net_conf).eval()
    x = torch.zeros(1, 1000)
    with torch.no_grad(), pytest.raises(RuntimeError, match='HIP device'):
        net(x, x, x, x)
    net.train()
    with torch.no_grad(), pytest.raises(NotImplementedError, match='eval'):
        net(x, x, x, x)
