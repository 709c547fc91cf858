"""Drop-in for the reference's Stage-2 inference entry point, scripts/test.py.

The command line is the same (test.py:172-208):

    python acoustic-echo-cancellation_amd/scripts/test.py \\
        --tt_list tt_list.txt --filename_list filename.txt --ckpt_dir exp \\
        [--model_file exp/models/best_loss.pt] [--est_path DIR]

So are the outputs (test.py:137-169):
- the data is read from the HDF5 file named on the FIRST line of tt_list,
  for every line. This reference quirk (test.py:138) is kept.
- outputs go to est_path/<basename(tt_list[i]) without '.ex'>/.
- each utterance k gets {k}_near_est.wav, {k}_near.wav, {k}_far.wav,
  {k}_mic.wav and {k}_echo.wav as 16 kHz PCM_16 (soundfile's default, see
  aec_amd.wavio).
- {k}_near_est.wav holds Little_net(mic=nearend_mic, ref=farend_speech,
  near=nearend_speech) at batch-1 semantics (test.py:157).

What differs is how the work is scheduled. Utterances are batched per GPU
call: the results are bit-identical to running them one at a time, which
`tests/test_gpu_parity.py` checks as batch invariance. Under torchrun, each
rank processes a length-balanced shard of the utterances and writes its own
files; the only collective is then a scalar sum of run
metrics. With `--gather`, the enhanced waveforms are gathered to rank 0 over
the process group (RCCL over xGMI, `shard.gather_to_root`) and rank 0
writes every file.

Extra flags (all optional):
- `--nlms` puts the FD-NLMS stage in front of the post-filter;
- `--streams` sets the utterances per GPU call;
- `--device` picks the GPU (default: LOCAL_RANK, the rank's bound GPU);
- `--gather` writes every file on rank 0 (waveforms gathered over RCCL).
"""
from __future__ import annotations

import argparse
import logging
import os
import pprint
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import h5lite, shard, wavio
from .configs import erb_conf, nlms_conf, speech_conf

# enhance(mic, ref, near, lengths[B][3] = (mic, ref, near) lengths) -> list of
# 1-D float32 outputs, one per row, each 256*(n_mic//256) samples
Enhancer = Callable[[np.ndarray, np.ndarray, np.ndarray, np.ndarray], List[np.ndarray]]


def get_logger(name, log_file=False):
    """scripts/utils/tools.py:11-22: same format; a file handler when log_file."""
    logger = logging.getLogger(name)
    logger.setLevel(logging.INFO)
    handler = logging.StreamHandler() if not log_file else logging.FileHandler(name)
    handler.setFormatter(logging.Formatter(fmt='%(asctime)s [%(pathname)s:%(lineno)s - %(levelname)s ] %(message)s',
                                           datefmt='%Y-%m-%d %H:%M:%S'))
    logger.addHandler(handler)
    return logger


def build_parser():
    p = argparse.ArgumentParser(description='Additioal configurations for testing',
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument('--tt_list', type=str, required=True, default='../examples/filelists/tt_list.txt',
                   help='Path to the list of testing files')
    p.add_argument('--filename_list', type=str, required=True, default='../examples/filelists/filename.txt')
    p.add_argument('--ckpt_dir', type=str, required=True, default='exp')
    p.add_argument('--model_file', type=str, default='./exp/models/best_loss.pt', help='Path to the model file')
    p.add_argument('--est_path', type=str, default='/data/lihaoming/datasets/synthetic/estimate',
                   help='Path to dump estimates')
    # gfx950 extras
    p.add_argument('--nlms', action='store_true', help='FD-NLMS linear AEC in front of the post-filter')
    p.add_argument('--streams', type=int, default=64, help='utterances per GPU call')
    p.add_argument('--device', type=int, default=None, help='GPU index (default: LOCAL_RANK or 0)')
    p.add_argument('--gather', action='store_true',
                   help='under torchrun: gather the enhanced waveforms to rank 0, which writes every file')
    return p


def _dist():
    """(rank, world); joins the torchrun process group when one is configured,
    with this rank bound to its LOCAL_RANK GPU (shard.init_process_group)."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world <= 1:
        return 0, 1
    import torch.distributed as dist
    shard.init_process_group()
    return dist.get_rank(), dist.get_world_size()


class Tester(object):
    """scripts/test.py:70-169."""

    def __init__(self, args, enhance: Optional[Enhancer] = None):
        self.sample_rate = speech_conf['sample_rate']
        self.model_file = args.model_file
        self.ckpt_dir = args.ckpt_dir
        self.est_path = args.est_path
        self.fimename_list = args.filename_list
        with open(args.tt_list, 'r') as f:
            self.tt_list = [line.strip() for line in f.readlines()]
        self.args = args
        self._enhance = enhance

    # -- the GPU enhancer: Little_net on this rank's device -------------------
    def _gpu_enhancer(self, logger, rank) -> Enhancer:
        import torch
        from .checkpoint import CheckPoint
        from .erb import EquivalentRectangularBandwidth
        from .little_net import Little_net
        local = self.args.device if self.args.device is not None else shard.local_rank()
        device = torch.device('cuda', local)
        net = Little_net(speech_conf, erb_conf['total_erb_bands'], nlms=nlms_conf if self.args.nlms else None)
        logger.info('backbone summary:\n{}'.format(net))
        param_count = sum(int(np.prod(p.shape)) for p in net.parameters())
        logger.info('Trainable parameter count: {:,d} -> {:.2f} MB\n'.format(param_count,
                                                                            param_count * 32 / 8 / (2 ** 20)))
        logger.info('Loading model from {}'.format(self.model_file))
        ckpt = CheckPoint().load(self.model_file, 'cpu')
        net.load_state_dict(ckpt.net_state_dict)
        net = net.to(device).eval()
        ERB = EquivalentRectangularBandwidth(erb_conf['nfreqs'], erb_conf['sample_rate'], erb_conf['total_erb_bands'],
                                             erb_conf['low_freq'], erb_conf['max_freq'])
        erb = torch.tensor(ERB.filters, dtype=torch.float32, device=device)

        def enhance(mic, ref, near, lengths):
            lengths = np.asarray(lengths, np.int64).reshape(len(mic), 3)
            with torch.no_grad():
                M, R, N = (torch.from_numpy(a).to(device, non_blocking=True) for a in (mic, ref, near))
                out, _ = net.forward_ragged(M, R, N, erb, lengths)
                out = out.cpu().numpy()
            return [out[b, :256 * (int(n) // 256)] for b, n in enumerate(lengths[:, 0])]

        return enhance

    def test(self):
        rank, world = _dist()
        os.makedirs(self.ckpt_dir, exist_ok=True)
        logger = get_logger(os.path.join(self.ckpt_dir, 'test.log' if world == 1 else f'test.rank{rank}.log'),
                            log_file=True)
        enhance = self._enhance or self._gpu_enhancer(logger, rank)
        with open(self.fimename_list) as f:                          # read but unused (test.py:130-131)
            f.readlines()
        pool = ThreadPoolExecutor(max_workers=8)
        n_utt = n_frames = 0
        gather = bool(getattr(self.args, 'gather', False)) and world > 1
        local = {}
        t0 = time.perf_counter()
        for i in range(len(self.tt_list)):
            reader = h5lite.File(self.tt_list[0])                    # test.py:138 reads tt_list[0] every time
            est_subdir = os.path.join(self.est_path, self.tt_list[i].split('/')[-1].replace('.ex', ''))
            os.makedirs(est_subdir, exist_ok=True)
            n = len(reader)
            lengths = [reader[str(k)]['nearend_speech'].shape[0] for k in range(n)]
            mine = shard.balanced_shards(lengths, world)[rank]
            mine.sort(key=lambda k: (-lengths[k], k))                # similar lengths share a call
            futs = []
            for s in range(0, len(mine), max(1, self.args.streams)):
                ks = mine[s:s + self.args.streams]
                egs = [self._load(reader, k) for k in ks]
                sig = ('nearend_mic', 'farend_speech', 'nearend_speech')     # mic, ref, near (test.py:157)
                lens = np.array([[len(e[key]) for key in sig] for e in egs], np.int64)
                rows = {key: np.zeros((len(ks), int(lens.max())), np.float32) for key in sig}
                for b, e in enumerate(egs):
                    for key in sig:
                        rows[key][b, :len(e[key])] = e[key]
                outs = enhance(rows['nearend_mic'], rows['farend_speech'], rows['nearend_speech'], lens)
                for k, e, out in zip(ks, egs, outs):
                    if gather:
                        local[k] = out
                    else:
                        futs.append(pool.submit(self._write, est_subdir, k, out, e))
                    n_utt += 1
                    n_frames += len(e['nearend_mic']) // 256 + 1
            if gather:
                merged = shard.gather_to_root(local)
                local = {}
                if merged is not None:
                    for k in sorted(merged):
                        futs.append(pool.submit(self._write, est_subdir, k, merged[k], self._load(reader, k)))
            for fu in futs:
                fu.result()
            reader.close()
        pool.shutdown()
        el = time.perf_counter() - t0
        tot_utt, tot_frames = shard.sum_over_ranks([n_utt, n_frames])
        el = shard.max_over_ranks(el)
        logger.info('enhanced {} utterances ({} frames) on {} rank(s) in {:.2f} s'.format(
            int(tot_utt), int(tot_frames), world, el))
        return int(tot_utt), int(tot_frames)

    @staticmethod
    def _load(reader, k):
        """ValidateDataset.__getitem__ (test.py:25-33) as the test loader delivers
        it: DataLoader(batch_size=1) with the DEFAULT collate (test.py:139; the
        padding collate_fn at :38-67 is not passed), so every signal keeps its
        stored length, and so do the WAVs written from it (:165-169)."""
        return h5lite.read_utterance(reader, k)

    def _write(self, est_subdir, k, out, e):
        sr = self.sample_rate
        wavio.write_wav(os.path.join(est_subdir, str(k) + '_near_est.wav'), out, sr)
        wavio.write_wav(os.path.join(est_subdir, str(k) + '_near.wav'), e['nearend_speech'], sr)
        wavio.write_wav(os.path.join(est_subdir, str(k) + '_far.wav'), e['farend_speech'], sr)
        wavio.write_wav(os.path.join(est_subdir, str(k) + '_mic.wav'), e['nearend_mic'], sr)
        wavio.write_wav(os.path.join(est_subdir, str(k) + '_echo.wav'), e['echo'], sr)


def main(argv=None):
    args = build_parser().parse_args(argv)
    get_logger(__name__).info('Arguments in command:\n{}'.format(pprint.pformat(vars(args))))
    Tester(args).test()


if __name__ == '__main__':
    main()
