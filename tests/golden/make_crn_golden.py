"""Generate the DCCRN golden vectors by importing and running the REFERENCE.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_crn_golden.py

For each case it builds the reference model (``network.dccrn.DCCRN``,
Stage2_lhm/scripts/network/dccrn.py:453, or
``scripts.network.dccrn2.DCCRN``, Stage2_lhm/scripts/network/dccrn2.py:10)
from a config derived from ``configs.net_conf`` (scripts/configs.py:29-46),
loads the seeded fixture weights of ``oracle/crn_oracle.make_weights`` through
the reference's own ``load_state_dict`` (so the weights never need to be
committed: they are regenerated from the seed by NumPy PCG64), puts it in
eval mode and runs one utterance (batch = 1) on CPU.  Stored per case: the
inputs, ``out_wav``, ``out_spec``, ``near_specs``, the decoder output (mask)
captured by a forward hook, the first encoder block's output and, for
dccrn.py, the loss.  Only data is written; no reference source is copied.
"""
import copy
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, '/root/reference/Stage2_lhm/scripts')
sys.path.insert(0, '/root/reference/Stage2_lhm')
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
sys.path.insert(0, os.path.join(REPO, 'oracle'))

from configs import net_conf                                  # noqa: E402  (reference)
from network.dccrn import DCCRN as DCCRN1                     # noqa: E402  (reference)
from scripts.network.dccrn2 import DCCRN as DCCRN2            # noqa: E402  (reference)
from aec_amd import synth                                     # noqa: E402  (ours: inputs only)
import crn_oracle                                             # noqa: E402  (ours: weights only)

torch.set_num_threads(8)

# (name, version, conf overrides, N, input seed, weight seed)
CASES = [
    ('v2E_2125', 2, {}, 2125, 11, 1),
    ('v2E_16000', 2, {}, 16000, 12, 1),
    ('v2C_bn_2125', 2, {'use_cbn': False, 'masking_mode': 'C'}, 2125, 13, 2),
    ('v2R_1000', 2, {'masking_mode': 'R'}, 1000, 14, 3),
    ('v1_2125', 1, {}, 2125, 15, 4),
    ('v2E_255', 2, {}, 255, 16, 1),
]


def run(name, version, over, n, seed, wseed):
    conf = copy.deepcopy(net_conf)
    conf.update(over)
    net = (DCCRN1 if version == 1 else DCCRN2)(conf)
    w = crn_oracle.make_weights(conf, version, wseed)
    missing, unexpected = net.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()}, strict=False)
    assert not unexpected, unexpected
    assert all(k.startswith(('stft.', 'istft.')) or k.endswith('num_batches_tracked') for k in missing), missing
    net.eval()
    cap = {}
    hooks = [net.decoder[-1].register_forward_hook(lambda m, i, o: cap.update(mask=o.detach().clone())),
             net.encoder[0].register_forward_hook(lambda m, i, o: cap.update(enc0=o.detach().clone()))]
    mic, far, near, echo = synth.scene(n, seed, return_echo=True)
    T = lambda a: torch.from_numpy(a)[None]
    with torch.no_grad():
        res = net(T(mic), T(far), T(near), T(echo))
    for h in hooks:
        h.remove()
    if version == 1:
        out_wav, out_spec, near_spec, loss = res
    else:
        out_spec, out_wav, near_spec = res
        loss = None
    arrays = dict(mic=mic, far=far, near=near, echo=echo, out_wav=out_wav[0].numpy(),
                  out_spec=out_spec[0].numpy(), near_spec=near_spec[0].numpy(),
                  mask=cap['mask'][0].numpy())
    if n <= 2125:
        arrays['enc0'] = cap['enc0'][0].numpy()
    if loss is not None:
        arrays['loss'] = np.float32(loss)
    np.savez_compressed(os.path.join(HERE, f'crn_{name}.npz'), **arrays)
    meta = dict(version=version, overrides=over, n=n, seed=seed, weight_seed=wseed,
                out_len=int(out_wav.shape[-1]), loss=None if loss is None else float(loss),
                out_rms=float(np.sqrt(np.mean(out_wav.numpy().astype(np.float64) ** 2))) if out_wav.numel() else 0.0)
    print(name, meta)
    return meta


def main():
    meta = {name: run(name, v, o, n, s, ws) for name, v, o, n, s, ws in CASES}
    with open(os.path.join(HERE, 'crn_meta.json'), 'w') as f:
        json.dump(meta, f, indent=1)


if __name__ == '__main__':
    main()
