"""Training-side mirrors of scripts/train1.py.

* ``TrainDataset`` / ``TrainDataset.collate_fn`` — train1.py:29-74: one HDF5
  file per utterance (root datasets ``nearend_speech``, ``nearend_mic``,
  ``farend_speech``, ``echo``), read with ``h5lite`` (h5py is absent); the
  batch zero-padded to the longest ``nearend_speech``.
* ``Adam`` — ``torch.optim.Adam`` (train1.py:153) with the update of a param
  group in one HIP launch (``aec_adam_step_multi``, include/aec_hip.h).  Same
  constructor, same ``state`` keys (``step``, ``exp_avg``, ``exp_avg_sq``), so
  its ``state_dict`` is interchangeable with torch's (the reference's
  ``CheckPoint`` stores ``optimizer.state_dict()``, train1.py:244-246).
* ``train_step`` — one iteration of ``Trainer.train`` (train1.py:199-218):
  forward on the padded batch, ``loss.backward()``, optional clipping
  (``clip_norm >= 0``), ``optimizer.step()``.

The forward / backward themselves are ``Little_net.forward`` in ``train()``
mode (``aec_train_forward`` / ``aec_train_backward``).
"""
from __future__ import annotations

import numpy as np
import torch
from torch.autograd.graph import increment_version

from . import _lib, h5lite

_KEYS = ('nearend_speech', 'nearend_mic', 'farend_speech', 'echo')


class TrainDataset(torch.utils.data.Dataset):
    """train1.py:29-41: item i = the four signals of HDF5 file dataset_path[i]."""

    def __init__(self, dataset_path):
        self.dataset_path = dataset_path

    def __getitem__(self, item):
        with h5lite.File(self.dataset_path[item]) as reader:
            return {k: np.array(reader[k]) for k in _KEYS}

    def __len__(self):
        return len(self.dataset_path)

    @staticmethod
    def collate_fn(data_list):
        """train1.py:43-74: every signal zero-padded to the longest
        ``nearend_speech`` of the batch; float32 tensors + ``n_samples``."""
        max_len = max(len(d['nearend_speech']) for d in data_list)
        out = {}
        for k in _KEYS:
            out[k] = torch.tensor(np.stack([np.pad(np.asarray(d[k], np.float32), (0, max_len - len(d[k])), 'constant')
                                            for d in data_list]), dtype=torch.float32)
        out['n_samples'] = max_len
        return out


_adam_handles = {}


def _adam_handle(dev):
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    h = _adam_handles.get(idx)
    if h is None:
        h = _adam_handles[idx] = _lib.Handle(idx)
    return h


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad = False, maximize = False) on the device:
    one ``aec_adam_step_multi`` launch per param group (and device)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False):
        if amsgrad:
            raise NotImplementedError('amsgrad (train1.py:153 passes amsgrad=False)')
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError('invalid Adam hyper-parameter')
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f'invalid betas {betas}')
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=False, differentiable=False,
                                      fused=None))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group['betas']
            per_dev = {}
            for p in group['params']:
                if p.grad is None:
                    continue
                if p.device.type != 'cuda' or p.dtype != torch.float32 or not p.is_contiguous():
                    raise RuntimeError('aec_amd.train.Adam updates contiguous float32 parameters on a HIP device')
                if p.grad.is_sparse:
                    raise RuntimeError('Adam does not support sparse gradients')
                st = self.state[p]
                if len(st) == 0:
                    st['step'] = torch.tensor(0.0)
                    st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st['step'] += 1
                per_dev.setdefault(p.device, []).append((p, p.grad.contiguous(), st))
            for dev, items in per_dev.items():
                h = _adam_handle(dev)
                with torch.cuda.device(dev):
                    # one launch for the group's tensors on this device (aec_adam_step_multi)
                    h.adam_step_multi([p.data_ptr() for p, _, _ in items], [g.data_ptr() for _, g, _ in items],
                                      [st['exp_avg'].data_ptr() for _, _, st in items],
                                      [st['exp_avg_sq'].data_ptr() for _, _, st in items],
                                      [p.numel() for p, _, _ in items], [int(st['step'].item()) for _, _, st in items],
                                      group['lr'], b1, b2, group['eps'], group['weight_decay'],
                                      torch.cuda.current_stream(dev).cuda_stream)
                # the kernel wrote the parameters through raw pointers: bump their version counters
                # as torch.optim.Adam's in-place ops do, so caches keyed on (data_ptr, _version) --
                # Little_net's weight upload -- see the step
                for p, _, _ in items:
                    increment_version(p)
        return loss


def train_step(net, egs, erb, optimizer, clip_norm=-1.0, device=None):
    """One iteration of Trainer.train (train1.py:199-218) on a collated batch
    ``egs``; returns the loss (a 0-d device tensor)."""
    device = torch.device(device) if device is not None else next(net.parameters()).device
    near = egs['nearend_speech'].to(device, non_blocking=True)
    mic = egs['nearend_mic'].to(device, non_blocking=True)
    far = egs['farend_speech'].to(device, non_blocking=True)
    optimizer.zero_grad()
    with torch.enable_grad():
        _, loss = net(mic, far, near, erb)
    loss.backward()
    if clip_norm >= 0.0:
        torch.nn.utils.clip_grad_norm_(net.parameters(), clip_norm)
    optimizer.step()
    return loss.detach()
