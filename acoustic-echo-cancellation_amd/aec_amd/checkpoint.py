"""Loader for the reference's `CheckPoint` files.

The reference saves its models with `torch.save(self)` on a
`utils.tools.CheckPoint` object (scripts/utils/tools.py:65-82). The object has
three attributes:
- `ckpt_info`: a dict;
- `net_state_dict`: an OrderedDict of tensors;
- `optim_state_dict`: a dict.

`scripts/test.py:122-124` then loads `ckpt.net_state_dict` into `Little_net`.

Loading such a pickle normally needs `weights_only=False`, which would
execute arbitrary code from the file. Here it goes through
`torch.load(weights_only=True)` instead. Only one extra global is allowed: a
plain attribute holder registered under the reference's name
`utils.tools.CheckPoint`. The unpickler builds that holder and fills its
`__dict__`; nothing from the file is imported or called. Plain state-dict
files and `{'net_state_dict': ...}` / `{'model': ...}` dicts load the same
way. The `module.` prefix of DataParallel checkpoints is stripped, as
scripts/train1.py:164-168 maps it.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Any, Dict, Optional

import torch


class CheckPoint(object):
    """Same surface as the reference's class (tools.py:65-82): ckpt_info,
    net_state_dict, optim_state_dict, and `load(filename, device)`.
    `save` is the training side and is out of scope."""

    def __init__(self, ckpt_info=None, net_state_dict=None, optim_state_dict=None):
        self.ckpt_info = ckpt_info
        self.net_state_dict = net_state_dict
        self.optim_state_dict = optim_state_dict

    def load(self, filename: str, device=None) -> 'CheckPoint':
        if not os.path.isfile(filename):
            raise FileNotFoundError('No checkpoint found at {}'.format(filename))
        obj = load_safely(filename, device)
        if isinstance(obj, _RefCheckPoint):
            d = obj.__dict__
            self.ckpt_info = d.get('ckpt_info')
            self.net_state_dict = d.get('net_state_dict')
            self.optim_state_dict = d.get('optim_state_dict')
        elif isinstance(obj, dict) and ('net_state_dict' in obj or 'model' in obj or 'state_dict' in obj):
            self.ckpt_info = obj.get('ckpt_info')
            self.net_state_dict = obj.get('net_state_dict', obj.get('model', obj.get('state_dict')))
            self.optim_state_dict = obj.get('optim_state_dict')
        elif isinstance(obj, dict) and all(torch.is_tensor(v) for v in obj.values()):
            self.ckpt_info, self.net_state_dict, self.optim_state_dict = None, obj, None
        else:
            raise ValueError(f'{filename}: not a CheckPoint, a checkpoint dict or a state_dict')
        self.net_state_dict = strip_module_prefix(self.net_state_dict)
        return self


class _RefCheckPoint(object):
    """Attribute holder the weights-only unpickler may build for the
    reference's `utils.tools.CheckPoint` (its pickle is NEWOBJ + BUILD with a
    plain attribute dict)."""


_RefCheckPoint.__module__ = 'utils.tools'
_RefCheckPoint.__qualname__ = 'CheckPoint'
_RefCheckPoint.__name__ = 'CheckPoint'


def load_safely(filename: str, device=None) -> Any:
    """torch.load with weights_only=True, allowing only the CheckPoint holder."""
    with torch.serialization.safe_globals([_RefCheckPoint]):
        return torch.load(filename, map_location=device if device is not None else 'cpu', weights_only=True)


def strip_module_prefix(sd: Optional[Dict[str, Any]]):
    if sd is None:
        return None
    if all(k.startswith('module.') for k in sd):
        return OrderedDict((k[len('module.'):], v) for k, v in sd.items())
    return sd
