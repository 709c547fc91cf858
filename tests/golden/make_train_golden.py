"""Golden vectors for the TRAINING step, made by
importing and running the REFERENCE in the build container:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_train_golden.py

What the reference's training loop does per iteration
(Stage2_lhm/scripts/train1.py:191-218):
* the batch is zero-padded to the longest utterance by
  ``TrainDataset.collate_fn`` (train1.py:43-74) — restated here with
  ``np.pad`` because train1.py itself imports h5py, which is absent;
* ``out_wav, loss = net(nearend_mic, farend_speech, nearend_speech, erb)``
  with the batch-GLOBAL normaliser of ERB.py:254-256 (one mean / std over the
  whole padded [B, N] tensor) and the batch-summed loss of ERB.py:318-323;
* ``loss.backward()``; no clipping (train_conf['clip_norm'] = -1);
* ``Adam(net.parameters(), lr=train_conf['lr'])`` ``.step()`` (train1.py:153).

Two iterations on two batches from ``torch.manual_seed(0)`` weights; stored:
inputs (float32, padded), lengths, loss, the 8 parameter gradients of each
iteration, and the parameters after each Adam step.  Only data is written;
no reference source is copied.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, '/root/reference/Stage2_lhm/scripts')
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))

from network.ERB import Little_net, EquivalentRectangularBandwidth   # noqa: E402  (reference)
from configs import speech_conf, erb_conf, train_conf                # noqa: E402  (reference)
from aec_amd import synth                                           # noqa: E402  (ours: inputs only)

torch.set_num_threads(4)
KEYS = ['gru1.weight_ih_l0', 'gru1.weight_hh_l0', 'gru1.bias_ih_l0', 'gru1.bias_hh_l0',
        'linear1.weight', 'linear1.bias', 'linear2.weight', 'linear2.bias']
BATCHES = [([8000, 6500, 7777], 200), ([5000, 5123], 300)]


def collate(lens, seed0):
    """train1.py:43-74: every signal zero-padded to max len(nearend_speech)."""
    mics, refs, nears = [], [], []
    for i, n in enumerate(lens):
        m, r, s = synth.scene(n, seed0 + i)
        mics.append(m); refs.append(r); nears.append(s)
    L = max(lens)
    pad = lambda xs: np.stack([np.pad(x, (0, L - len(x))) for x in xs]).astype(np.float32)
    return pad(mics), pad(refs), pad(nears)


def main():
    torch.manual_seed(0)
    net = Little_net(speech_conf, erb_conf['total_erb_bands'])
    net.train()
    erb = EquivalentRectangularBandwidth(erb_conf['nfreqs'], erb_conf['sample_rate'],
                                         erb_conf['total_erb_bands'], erb_conf['low_freq'],
                                         erb_conf['max_freq']).filters
    erb_t = torch.tensor(erb, dtype=torch.float32)
    lr = train_conf['lr']
    opt = torch.optim.Adam([{'params': net.parameters()}], lr=lr, amsgrad=False)
    names = [k for k, _ in net.named_parameters()]
    assert names == KEYS, names
    arrays, meta = {}, {'lr': lr, 'betas': [0.9, 0.999], 'eps': 1e-8, 'iters': []}
    for it, (lens, seed0) in enumerate(BATCHES):
        mic, ref, near = collate(lens, seed0)
        opt.zero_grad()
        with torch.enable_grad():
            out, loss = net(torch.from_numpy(mic), torch.from_numpy(ref), torch.from_numpy(near), erb_t)
        loss.backward()
        arrays[f'mic{it}'], arrays[f'ref{it}'], arrays[f'near{it}'] = mic, ref, near
        arrays[f'lens{it}'] = np.array(lens, np.int64)
        arrays[f'loss{it}'] = np.float32(loss.item())
        arrays[f'out_head{it}'] = out.detach()[:, :1024].numpy()
        for k, p in net.named_parameters():
            arrays[f'grad{it}/{k}'] = p.grad.detach().numpy().copy()
        opt.step()
        for k, p in net.named_parameters():
            arrays[f'param{it}/{k}'] = p.detach().numpy().copy()
        meta['iters'].append(dict(lens=lens, seed0=seed0, loss=float(loss.item()),
                                  grad_norm=float(torch.sqrt(sum((p.grad.double() ** 2).sum()
                                                                 for p in net.parameters())))))
        print(it, lens, float(loss), meta['iters'][-1]['grad_norm'])
    np.savez_compressed(os.path.join(HERE, 'train.npz'), **arrays)
    with open(os.path.join(HERE, 'train_meta.json'), 'w') as f:
        json.dump(meta, f, indent=1)


if __name__ == '__main__':
    main()
