"""Host-side checks that need no GPU: the drop-in module's construction,
state_dict compatibility, ERB class, and that the C-ABI library loads and
exports every symbol include/aec_hip.h declares."""
import ctypes
import os
import re
import sys

import numpy as np
import torch

from conftest import PARAM_KEYS, REPO


def test_erb_class_bit_exact(golden_erb):
    from aec_amd import EquivalentRectangularBandwidth, erb_conf
    e = EquivalentRectangularBandwidth(erb_conf['nfreqs'], erb_conf['sample_rate'], erb_conf['total_erb_bands'],
                                       erb_conf['low_freq'], erb_conf['max_freq']).filters
    assert e.dtype == np.float64
    assert np.array_equal(e, golden_erb)


def test_little_net_seed0_init_matches_reference(golden_weights):
    """Same module order + init scheme as ERB.py:204-229 -> same weights."""
    import aec_amd
    torch.manual_seed(0)
    net = aec_amd.Little_net(aec_amd.speech_conf, 32)
    sd = net.state_dict()
    for k in PARAM_KEYS:
        assert torch.equal(sd[k], torch.from_numpy(golden_weights[k])), k


def test_state_dict_keys_and_buffers(golden_weights):
    import aec_amd
    net = aec_amd.Little_net(aec_amd.speech_conf, 32)
    sd = net.state_dict()
    expected = set(PARAM_KEYS) | {'cpx_stft.weight', 'istft.weight', 'istft.window', 'istft.enframe'}
    assert set(sd.keys()) == expected
    assert tuple(sd['cpx_stft.weight'].shape) == (514, 1, 512)
    assert tuple(sd['istft.weight'].shape) == (514, 1, 512)
    assert tuple(sd['istft.window'].shape) == (1, 512, 1)
    assert tuple(sd['istft.enframe'].shape) == (512, 1, 512)
    rows = golden_weights['stft_rows']
    assert np.abs(sd['cpx_stft.weight'][rows, 0].numpy() - golden_weights['stft_weight_rows']).max() < 1e-6
    assert np.abs(sd['istft.weight'][rows, 0].numpy() - golden_weights['istft_weight_rows']).max() < 1e-7
    # strict reload of its own state_dict (the reference does load_state_dict strict, test.py:124)
    net.load_state_dict(sd, strict=True)
    assert sum(p.numel() for p in net.parameters()) == 12544      # numParams (tools.py:25-27)


def test_weights_blob_order(golden_weights):
    import aec_amd
    net = aec_amd.Little_net(aec_amd.speech_conf, 32)
    sd = net.state_dict()
    for k in PARAM_KEYS:
        sd[k] = torch.from_numpy(golden_weights[k])
    net.load_state_dict(sd)
    blob = net.weights_blob()
    exp = np.concatenate([golden_weights[k].reshape(-1) for k in PARAM_KEYS])
    assert blob.dtype == np.float32 and np.array_equal(blob, exp)


def test_clib_exports_every_declared_symbol():
    from aec_amd import _lib
    hdr = open(os.path.join(REPO, 'include', 'aec_hip.h')).read()
    declared = set(re.findall(r'^\s*(?:[A-Za-z_][\w\s\*]*?)\b(aec_\w+)\s*\(', hdr, re.M))
    assert declared == set(_lib.EXPORTS), declared ^ set(_lib.EXPORTS)
    lib = _lib.load()
    for s in declared:
        assert hasattr(lib, s), s
    # pure host helpers (no GPU needed): framing integers and the weights count
    for n in [1, 255, 256, 513, 16000, 160000]:
        assert lib.aec_num_frames(n) == n // 256 + 1
        assert lib.aec_out_len(n) == 256 * (n // 256)
    assert lib.aec_weights_count(32) == 12544
    assert lib.aec_weights_count(16) == 0


AB_KNOBS = ('AEC_MOM_CFG', 'AEC_MOM_GRID', 'AEC_GRU_MODE', 'AEC_GRU_WMAP', 'AEC_NLMS_PRIO', 'AEC_NLMS_ERB', 'AEC_FUSED_MODE',
            'AEC_CRN_ENC_FR', 'AEC_CRN_SPLITK', 'CRN_PERSIST_RA', 'AEC_CRN_ENC_MX_RERUN', 'CRN_DEC_FUSE',
            'CRN_GEMM_XCD', 'CRN_GEMM_DMA', 'CRN_GEMM_BIG', 'CRN_GEMM_SQ', 'CRN_GEMM_RB64', 'CRN_GEMM_MODE',
            'CRN_GEMM_PIPE', 'CRN_STEP_MODE', 'CRN_STEP_CFG', 'CRN_MX_STEP_MODE', 'AEC_CRN_PERSIST_WAVES')


def test_product_library_reads_only_mode_knobs():
    """The product libaec_hip.so is not an A/B build: none of the timing-only /
    work-skipping knob names (csrc/aec_knobs.h AEC_AB_KNOB) is in the binary,
    and every AEC_* / CRN_* environment name it holds is a listed mode knob."""
    from aec_amd import _lib
    info = _lib.build_info()
    assert info['arch'] == 'gfx950' and info['ab_knobs'] is False, info
    blob = open(_lib.LIB_PATH, 'rb').read()
    for k in AB_KNOBS:
        assert k.encode() + b'\0' not in blob, k
    names = set(m.decode() for m in re.findall(rb'\0((?:AEC|CRN)_[A-Z0-9_]+)\0', blob))
    names -= {'AEC_OK'}
    assert names <= set(info['mode_knobs']), names - set(info['mode_knobs'])
    assert 'AEC_CRN_GRAPH' in info['mode_knobs']


def test_product_path_does_not_import_oracle():
    pkg = os.path.join(REPO, 'acoustic-echo-cancellation_amd')
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(('.py', '.hip', '.h', '.cpp')):
                src = open(os.path.join(root, f)).read()
                assert 'aec_oracle' not in src and 'crn_oracle' not in src and 'oracle/' not in src, f


def test_cpu_tensors_fail_loudly(golden_erb):
    import aec_amd
    import pytest
    net = aec_amd.Little_net(aec_amd.speech_conf, 32).eval()
    x = torch.zeros(1, 1000)
    with torch.no_grad(), pytest.raises(RuntimeError, match='HIP device'):
        net(x, x, x, torch.tensor(golden_erb, dtype=torch.float32))


def test_erb_device_tables_match_dense(golden_erb):
    """The balanced ERB schedule and the transpose table the kernels use
    reproduce the reference's dense products mags @ erb and est @ erb^T."""
    from aec_amd import _lib
    rng = np.random.default_rng(0)
    erb32 = golden_erb.astype(np.float32)
    for _ in range(5):
        mags = rng.uniform(0, 3, 257).astype(np.float32)
        est = rng.uniform(0, 2, 32).astype(np.float32)
        bands, gains, L, conflicts = _lib.erb_tables_check(erb32, mags, est)
        assert L == 32                                   # 483 nnz over 16 lanes, <= 32 entries each
        assert conflicts <= 8                            # bank-residue matching of the schedule
        ref_b = mags.astype(np.float64) @ erb32.astype(np.float64)
        ref_g = est.astype(np.float64) @ erb32.T.astype(np.float64)
        assert np.abs(bands - ref_b).max() <= 1e-5 * np.abs(ref_b).max()
        assert np.abs(gains - ref_g).max() <= 1e-5 * np.abs(ref_g).max()
    # a filterbank with a bin in 3 bands is refused (UNSUPPORTED), not silently wrong
    bad = erb32.copy()
    bad[100, :3] = 1.0
    import pytest
    with pytest.raises(RuntimeError, match='UNSUPPORTED'):
        _lib.erb_tables_check(bad, mags, est)


def test_bench_refuses_timing_only_knobs(monkeypatch):
    """bench.py records every AEC_* / CRN_* variable and the library's build
    description, and refuses to produce a line when a timing-only (A/B build)
    or test-only knob is set (a driver line must show it ran the
    defaults)."""
    import importlib
    import pytest
    sys.path.insert(0, REPO)
    bench = importlib.import_module('bench')
    for k in list(os.environ):
        if k.startswith(('AEC_', 'CRN_')):
            monkeypatch.delenv(k)
    prov = bench.knob_provenance()
    assert prov['env'] == {} and prov['defaults'] is True and 'ab_knobs=off' in prov['build_info']
    monkeypatch.setenv('AEC_CRN_GRAPH', '1')                    # a tested mode: recorded, not refused
    prov = bench.knob_provenance()
    assert prov['env'] == {'AEC_CRN_GRAPH': '1'} and prov['defaults'] is False and prov['unknown_names'] == []
    for k in ('AEC_MOM_CFG', 'AEC_CRN_PERSIST_STALL'):
        monkeypatch.setenv(k, '9')
        with pytest.raises(SystemExit):
            bench.knob_provenance()
        monkeypatch.delenv(k)
