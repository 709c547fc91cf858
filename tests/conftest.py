import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
sys.path.insert(0, os.path.join(REPO, 'oracle'))
GOLDEN = os.path.join(REPO, 'tests', 'golden')

PARAM_KEYS = ['gru1.weight_ih_l0', 'gru1.weight_hh_l0', 'gru1.bias_ih_l0', 'gru1.bias_hh_l0',
              'linear1.weight', 'linear1.bias', 'linear2.weight', 'linear2.bias']


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a HIP device (MI355X)')


@pytest.fixture(scope='session')
def golden_weights():
    return dict(np.load(os.path.join(GOLDEN, 'weights.npz')))


@pytest.fixture(scope='session')
def golden_erb():
    return np.load(os.path.join(GOLDEN, 'erb.npy'))


def golden_case(name):
    return dict(np.load(os.path.join(GOLDEN, name + '.npz')))


CASES = ['case_255_1', 'case_256_2', 'case_513_3', 'case_16000_4', 'case_16123_5', 'case_16000_6']


@pytest.fixture(scope='session')
def gpu_net(golden_weights):
    """Little_net on cuda:0 loaded with the golden (reference seed-0) weights."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    import aec_amd
    net = aec_amd.Little_net(aec_amd.speech_conf, 32).eval()
    sd = net.state_dict()
    for k in PARAM_KEYS:
        sd[k] = torch.from_numpy(golden_weights[k])
    net.load_state_dict(sd, strict=True)
    return net.to('cuda:0')


# ---------------------------------------------------------------------------
# Parity margins: every reduced-precision bar goes through margin(), which
# asserts the bar and records the observed value, so a run leaves the
# observed-error vs bar table (gpurun_out/parity_margins.json) that the bars
# are sized from (about 1.5-2x the largest observed error).
# ---------------------------------------------------------------------------
_MARGINS = []


def margin(name, value, bar):
    value = float(value)
    test = os.environ.get('PYTEST_CURRENT_TEST', '').split(' ')[0]
    _MARGINS.append(dict(test=test, check=name, observed=value, bar=float(bar),
                         headroom=(float(bar) / value) if value > 0 else None))
    print(f'[margin] {name}: observed {value:.4g} bar {bar:.4g}')
    assert value <= bar, f'{name}: {value} > bar {bar}'


def pytest_sessionfinish(session, exitstatus):
    if not _MARGINS:
        return
    import json
    out = os.path.join(REPO, 'gpurun_out')
    try:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, 'parity_margins.json'), 'w') as f:
            json.dump(_MARGINS, f, indent=1)
    except OSError:
        pass
