"""Golden vectors for signals of DIFFERENT stored lengths, made by importing
and running the REFERENCE (build container only; it reads /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_siglens_golden.py

scripts/test.py:139 loads the HDF5 groups with DataLoader(batch_size=1) and
the DEFAULT collate (the padding collate_fn at test.py:38-67 is not passed),
so nearend_mic / farend_speech / nearend_speech reach
``Little_net.forward`` (ERB.py:252-334) at their own stored lengths: each is
normalised over its own samples (ERB.py:254-256) and zero-padded by its own
ConvSTFT (attention_ccrn.py:48).  The forward combines them frame by frame
(ERB.py:287-290, 318-323), so it runs when the three share N//256 + 1 frames
and raises otherwise.  This script records both behaviours:

* ``siglens.npz``: two cases with unequal lengths and equal frame counts
  (ref / near shorter than mic; ref longer than mic), inputs + the
  reference's out_wav and loss;
* ``siglens_meta.json``: the lengths, and the exception type the reference
  raises on a frame-count mismatch.

Uses the seed-0 weights of make_golden.py (same init).  Only data is written.
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
from configs import speech_conf, erb_conf                           # noqa: E402  (reference)
from aec_amd import synth                                           # noqa: E402  (ours: inputs only)

torch.set_num_threads(4)
CASES = [(16123, 16000, 15900, 200), (9000, 9200, 8970, 201)]      # (n_mic, n_ref, n_near, seed)


def main():
    torch.manual_seed(0)
    net = Little_net(speech_conf, erb_conf['total_erb_bands']).eval()
    erb = EquivalentRectangularBandwidth(erb_conf['nfreqs'], erb_conf['sample_rate'],
                                         erb_conf['total_erb_bands'], erb_conf['low_freq'],
                                         erb_conf['max_freq']).filters
    erb_t = torch.tensor(erb, dtype=torch.float32)
    w = np.load(os.path.join(HERE, 'weights.npz'))
    for k, v in net.state_dict().items():
        if k in w.files:
            assert np.array_equal(v.numpy(), w[k]), k        # the same weights as the other goldens
    arrays, meta = {}, {'cases': []}
    T = lambda a: torch.from_numpy(a)[None]
    for i, (nm, nr, nn_, seed) in enumerate(CASES):
        n = max(nm, nr, nn_)
        mic, ref, near = synth.scene(n, seed)
        mic, ref, near = mic[:nm], ref[:nr], near[:nn_]
        with torch.no_grad():
            out, loss = net(T(mic), T(ref), T(near), erb_t)
        arrays.update({f'mic{i}': mic, f'ref{i}': ref, f'near{i}': near, f'out{i}': out[0].numpy(),
                       f'loss{i}': np.float32(loss)})
        meta['cases'].append(dict(n_mic=nm, n_ref=nr, n_near=nn_, seed=seed, out_len=int(out.shape[-1]),
                                  loss=float(loss)))
    # frame-count mismatch: ref one hop longer than mic
    mic, ref, near = synth.scene(4000, 202)
    try:
        with torch.no_grad():
            net(T(mic[:3000]), T(ref[:3300]), T(near[:3000]), erb_t)
        meta['mismatch'] = 'no exception'
    except Exception as e:        # noqa: BLE001 — the type is the datum
        meta['mismatch'] = type(e).__name__
    np.savez_compressed(os.path.join(HERE, 'siglens.npz'), **arrays)
    with open(os.path.join(HERE, 'siglens_meta.json'), 'w') as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == '__main__':
    main()
