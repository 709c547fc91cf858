"""The test.py-compatible CLI end to end on the GPU: HDF5 set -> reference-style
CheckPoint -> Little_net on the HIP path -> PCM16 WAV tree, checked against
the oracle: the PCM16 difference is within the 1e-4 RMS waveform bar
(3.3 LSB RMS) and a few LSB at most (float differences near rounding
boundaries flip the last bit)."""
import os

import numpy as np
import pytest
import torch

import aec_oracle as O
from aec_amd import wavio
from aec_amd.tester import Tester as _Tester, build_parser
from conftest import PARAM_KEYS
from test_cli_io import LENS, _make_set, _save_reference_style

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('nlms', [False, True])
def test_cli_gpu_end_to_end(tmp_path, golden_weights, golden_erb, nlms):
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    utts, lst, fl = _make_set(tmp_path, seed=300)
    ck = str(tmp_path / 'best_loss.pt')
    import aec_amd
    sd = aec_amd.Little_net(aec_amd.speech_conf, 32).state_dict()      # all 12 keys, as net.state_dict() saves
    for key in PARAM_KEYS:
        sd[key] = torch.from_numpy(golden_weights[key])
    _save_reference_style(ck, sd, {'cur_epoch': 0})
    argv = ['--tt_list', lst, '--filename_list', fl, '--ckpt_dir', str(tmp_path / 'exp'),
            '--model_file', ck, '--est_path', str(tmp_path / 'est'), '--streams', '4']
    args = build_parser().parse_args(argv + (['--nlms'] if nlms else []))
    n_utt, _ = _Tester(args).test()
    assert n_utt == 2 * len(LENS)
    erb = golden_erb.astype(np.float32)
    cfg = dict(taps=4, mu=0.3, beta=0.5, delta=1e-4) if nlms else None
    for k, n in enumerate(LENS):
        est, _ = wavio.read_wav(str(tmp_path / 'est' / 'test' / f'{k}_near_est.wav'))
        assert est.shape == (256 * (n // 256),)
        o, _ = O.aec_forward(utts[k]['nearend_mic'], utts[k]['farend_speech'], utts[k]['nearend_speech'],
                             erb, golden_weights, nlms_cfg=cfg)
        if est.size:
            diff = wavio.pcm16(o).astype(int) - (est * 32768).astype(int)
            assert np.sqrt(np.mean(diff.astype(float) ** 2)) <= 1e-4 * 32767
            assert np.abs(diff).max() <= 8
