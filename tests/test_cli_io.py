"""§8(f) rows 1-2 on CPU: the test.py-compatible CLI plumbing, PCM16 WAV
I/O, and the safe CheckPoint loader.

The GPU enhancer is replaced here by the float64 oracle. The oracle is the
checker, not the product. This lets the file tree, batching, padding and
sharding logic run without a device. tests/test_gpu_cli.py runs the real
HIP path through the same CLI.
"""
import os
import socket
import sys
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import aec_oracle as O
from aec_amd import h5lite, wavio
from aec_amd.checkpoint import CheckPoint
from aec_amd.tester import Tester as _Tester, build_parser
from conftest import GOLDEN, PARAM_KEYS


# ---------------------------------------------------------------- WAV -------
def test_pcm16_matches_libsndfile_rule():
    x = np.array([0.0, 1.0, -1.0, 0.5, -0.5, 1.5 / 32767, 2.5 / 32767, 1e-9, 1.0 + 1.0 / 32767], np.float32)
    s = wavio.pcm16(x)
    # lrintf(x * 0x7FFF): ties to even (1.5 -> 2, 2.5 -> 2); 32768 wraps to -32768 (no clipping)
    assert s.tolist() == [0, 32767, -32767, 16384, -16384, 2, 2, 0, -32768]
    assert wavio.pcm16(x, clip=True)[-1] == 32767


def test_wav_roundtrip_and_header(tmp_path):
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(16001) * 0.2).astype(np.float32)
    p = str(tmp_path / 'a.wav')
    wavio.write_wav(p, x, 16000)
    raw = open(p, 'rb').read()
    assert raw[:4] == b'RIFF' and raw[8:16] == b'WAVEfmt ' and raw[36:40] == b'data'
    assert len(raw) == 44 + 2 * len(x)
    y, sr = wavio.read_wav(p)
    assert sr == 16000 and y.shape == x.shape
    assert np.array_equal((y * 32768).astype(np.int64), wavio.pcm16(x).astype(np.int64))


# ---------------------------------------------------------- checkpoint ------
def _save_reference_style(path, sd, info):
    """Write a pickle exactly as the reference does (tools.py:71-72:
    torch.save(self) on a utils.tools.CheckPoint), using a stand-in module
    registered only for the duration of the save."""
    m = types.ModuleType('utils.tools')
    pkg = types.ModuleType('utils')
    pkg.tools = m

    class CheckPointRef(object):
        def __init__(self, a, b, c):
            self.ckpt_info, self.net_state_dict, self.optim_state_dict = a, b, c

    CheckPointRef.__module__, CheckPointRef.__qualname__, CheckPointRef.__name__ = 'utils.tools', 'CheckPoint', 'CheckPoint'
    m.CheckPoint = CheckPointRef
    saved = {k: sys.modules.get(k) for k in ('utils', 'utils.tools')}
    sys.modules['utils'], sys.modules['utils.tools'] = pkg, m
    try:
        torch.save(CheckPointRef(info, sd, {'state': {}, 'param_groups': [{'lr': 1e-5, 'params': [0, 1]}]}), path)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def test_checkpoint_reference_pickle_loads_weights_only(tmp_path, golden_weights):
    sd = {k: torch.from_numpy(golden_weights[k]) for k in PARAM_KEYS}
    p = str(tmp_path / 'best_loss.pt')
    _save_reference_style(p, sd, {'cur_epoch': 4, 'cur_iter': 10, 'cv_loss': 0.25, 'best_loss': 0.25})
    assert 'utils' not in sys.modules or not hasattr(sys.modules.get('utils'), 'tools')
    c = CheckPoint().load(p, 'cpu')
    assert c.ckpt_info['cur_epoch'] == 4
    assert set(c.net_state_dict) == set(PARAM_KEYS)
    for k in PARAM_KEYS:
        assert torch.equal(c.net_state_dict[k], sd[k])
    assert c.optim_state_dict['param_groups'][0]['lr'] == 1e-5


def test_checkpoint_plain_and_dataparallel(tmp_path):
    sd = {'module.gru1.weight_ih_l0': torch.ones(2), 'module.linear1.bias': torch.zeros(3)}
    p = str(tmp_path / 'sd.pt')
    torch.save(sd, p)
    c = CheckPoint().load(p)
    assert list(c.net_state_dict) == ['gru1.weight_ih_l0', 'linear1.bias'] and c.ckpt_info is None
    torch.save({'net_state_dict': {'a': torch.ones(1)}, 'ckpt_info': {'x': 1}}, p)
    assert CheckPoint().load(p).ckpt_info == {'x': 1}
    with pytest.raises(FileNotFoundError):
        CheckPoint().load(str(tmp_path / 'missing.pt'))


def test_checkpoint_refuses_arbitrary_globals(tmp_path):
    class Evil(object):
        def __reduce__(self):
            return (os.system, ('true',))
    p = str(tmp_path / 'evil.pt')
    torch.save({'net_state_dict': Evil()}, p)
    with pytest.raises(Exception):
        CheckPoint().load(p)


# ---------------------------------------------------------------- CLI -------
LENS = [16123, 513, 40000, 255, 30001, 9000, 16000]


def _make_set(tmp_path, seed=0):
    from aec_amd import synth
    utts = []
    for i, n in enumerate(LENS):
        mic, ref, near = synth.scene(n, seed + i)
        echo = (mic - near)[: n - (i % 3) * 17]                   # some echo rows shorter: kept as stored
        # some ref / near rows shorter than the mic, same frame count (N//256 + 1): each signal is
        # normalised over its own stored length, as the reference's default collate delivers it
        d = min(17 * (i % 2), n % 256)
        ref, near = ref[:n - d], near[:n - (d // 2)]
        utts.append({'nearend_speech': near, 'nearend_mic': mic, 'farend_speech': ref, 'echo': echo})
    h5 = str(tmp_path / 'test.ex')
    h5lite.write_utterances(h5, utts)
    lst = tmp_path / 'tt_list.txt'
    lst.write_text(h5 + '\n' + str(tmp_path / 'second.ex'))      # 2 lines: the quirk reads line 1 twice
    fl = tmp_path / 'filename.txt'
    fl.write_text('\n'.join(str(i) for i in range(len(LENS))))
    return utts, str(lst), str(fl)


def _oracle_enhancer(weights, erb):
    def enhance(mic, ref, near, lengths):
        return [O.little_net_forward(mic[b, :l[0]], ref[b, :l[1]], near[b, :l[2]], erb, weights)[0].astype(np.float32)
                for b, l in enumerate(np.asarray(lengths).reshape(-1, 3))]
    return enhance


def _args(tmp_path, lst, fl, streams=3, extra=()):
    return build_parser().parse_args(['--tt_list', lst, '--filename_list', fl, '--ckpt_dir',
                                      str(tmp_path / 'exp'), '--est_path', str(tmp_path / 'est'),
                                      '--streams', str(streams), *extra])


def test_cli_file_tree_and_contents(tmp_path, golden_weights, golden_erb):
    utts, lst, fl = _make_set(tmp_path)
    enh = _oracle_enhancer(golden_weights, golden_erb.astype(np.float32))
    n_utt, n_frames = _Tester(_args(tmp_path, lst, fl), enhance=enh).test()
    assert n_utt == 2 * len(LENS) and n_frames == 2 * sum(n // 256 + 1 for n in LENS)
    for sub in ['test', 'second']:                                   # est_path/<basename minus .ex>
        d = tmp_path / 'est' / sub
        names = sorted(os.listdir(d))
        assert names == sorted(f'{k}_{s}.wav' for k in range(len(LENS))
                               for s in ['near_est', 'near', 'far', 'mic', 'echo'])
        for k, n in enumerate(LENS):
            est, sr = wavio.read_wav(str(d / f'{k}_near_est.wav'))
            assert sr == 16000 and est.shape == (256 * (n // 256),)
            o, _ = O.little_net_forward(utts[k]['nearend_mic'], utts[k]['farend_speech'],
                                        utts[k]['nearend_speech'], golden_erb.astype(np.float32), golden_weights)
            if est.size:
                assert np.abs(wavio.pcm16(o).astype(int) - (est * 32768).astype(int)).max() <= 1
            # every input signal is written back at its stored length, byte for byte (test.py:165-169:
            # default collate, no padding)
            for key, suf in (('echo', 'echo'), ('nearend_speech', 'near'), ('farend_speech', 'far'),
                             ('nearend_mic', 'mic')):
                raw = open(str(d / f'{k}_{suf}.wav'), 'rb').read()
                x = utts[k][key]
                assert len(raw) == 44 + 2 * len(x)
                assert raw[44:] == wavio.pcm16(x).astype('<i2').tobytes()
    assert (tmp_path / 'exp' / 'test.log').exists()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, tmp, lst, fl, weights, erb, q, extra=()):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import pathlib
        tmp = pathlib.Path(tmp)
        res = _Tester(_args(tmp, lst, fl, streams=2, extra=extra), enhance=_oracle_enhancer(weights, erb)).test()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('gather', [False, True], ids=['per-rank-writes', 'gather-to-rank0'])
def test_cli_two_ranks_gloo(tmp_path, golden_weights, golden_erb, gather):
    utts, lst, fl = _make_set(tmp_path, seed=50)
    extra = ('--gather',) if gather else ()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    erb = golden_erb.astype(np.float32)
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, str(tmp_path), lst, fl, golden_weights, erb, q, extra))
          for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    # both ranks report the job totals (metric all-reduce); every file written once
    assert res[0][1] == res[1][1] == (2 * len(LENS), 2 * sum(n // 256 + 1 for n in LENS))
    names = os.listdir(tmp_path / 'est' / 'test')
    assert len(names) == 5 * len(LENS) and len(set(names)) == len(names)
    # the estimates are the single-utterance results whichever rank produced them
    for k in (0, 2, 6):
        est, _ = wavio.read_wav(str(tmp_path / 'est' / 'test' / f'{k}_near_est.wav'))
        o, _ = O.little_net_forward(utts[k]['nearend_mic'], utts[k]['farend_speech'], utts[k]['nearend_speech'],
                                    erb, golden_weights)
        assert np.abs(wavio.pcm16(o).astype(int) - (est * 32768).astype(int)).max() <= 1
