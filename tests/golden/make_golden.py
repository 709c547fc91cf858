"""Generate the golden vectors by importing and running the REFERENCE.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it does:
* builds ``network.ERB.Little_net(speech_conf, 32)`` after
  ``torch.manual_seed(0)`` (the reference's own init: orthogonal GRU,
  kaiming linears, ERB.py:204-229) and saves its 8 parameter tensors to
  ``weights.npz`` (the STFT buffers are closed-form; only spot rows of them
  are kept, to pin the closed forms);
* builds ``EquivalentRectangularBandwidth(**erb_conf).filters`` -> ``erb.npy``;
* runs ``net(mic, ref, near, erb)`` at batch=1 on CPU (scripts/test.py:157
  semantics) for seeded synthetic scenes and stores inputs, outputs and the
  intermediates captured by forward hooks on the reference's own sub-modules
  (cpx_stft, gru1, linear2, istft) in ``case_<N>.npz``;
* for a 10 s utterance stores only the output summary (rms, head/tail
  samples, loss) plus a SHA-256 of the regenerated inputs;
* for a ragged 3-utterance set stores the per-utterance (batch=1) outputs and
  the RMS difference of the reference's *batched* call (documents the
  batch-global normaliser hazard).
Only data is written here; no reference source is copied.
"""
import hashlib
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


def build_net():
    torch.manual_seed(0)
    net = Little_net(speech_conf, erb_conf['total_erb_bands']).eval()
    return net


def run_case(net, erb_t, mic, ref, near):
    cap = {}
    specs = []
    hooks = [
        net.cpx_stft.register_forward_hook(lambda m, i, o: specs.append(o.detach().clone())),
        net.gru1.register_forward_hook(lambda m, i, o: cap.update(gru_in=i[0].detach().clone(),
                                                                  gru_out=o[0].detach().clone())),
        net.linear2.register_forward_hook(lambda m, i, o: cap.update(mask=torch.sigmoid(o).detach().clone())),
        net.istft.register_forward_hook(lambda m, i, o: cap.update(out_spec=i[0].detach().clone())),
    ]
    with torch.no_grad():
        out, loss = net(torch.from_numpy(mic)[None], torch.from_numpy(ref)[None],
                        torch.from_numpy(near)[None], erb_t)
    for h in hooks:
        h.remove()
    near_s, mic_s, ref_s = specs          # call order ERB.py:262-264
    return out[0].numpy(), float(loss), cap, (mic_s[0].numpy(), ref_s[0].numpy(), near_s[0].numpy())


def main():
    net = build_net()
    sd = {k: v.numpy() for k, v in net.state_dict().items()}
    params = {k: sd[k] for k in ['gru1.weight_ih_l0', 'gru1.weight_hh_l0', 'gru1.bias_ih_l0',
                                 'gru1.bias_hh_l0', 'linear1.weight', 'linear1.bias',
                                 'linear2.weight', 'linear2.bias']}
    rows = np.array([0, 1, 2, 100, 255, 256, 257, 258, 300, 511, 512, 513])
    np.savez(os.path.join(HERE, 'weights.npz'),
             **params,
             stft_rows=rows,
             stft_weight_rows=sd['cpx_stft.weight'][rows, 0, :],
             istft_weight_rows=sd['istft.weight'][rows, 0, :],
             istft_window=sd['istft.window'][0, :, 0])
    erb = EquivalentRectangularBandwidth(erb_conf['nfreqs'], erb_conf['sample_rate'],
                                         erb_conf['total_erb_bands'], erb_conf['low_freq'],
                                         erb_conf['max_freq']).filters
    np.save(os.path.join(HERE, 'erb.npy'), erb)
    erb_t = torch.tensor(erb, dtype=torch.float32)          # scripts/test.py:111

    meta = {}
    for n, seed, dt in [(255, 1, True), (256, 2, True), (513, 3, True),
                        (16000, 4, True), (16123, 5, True), (16000, 6, False)]:
        mic, ref, near = synth.scene(n, seed, double_talk=dt)
        if not dt:
            near = near + np.float32(1e-3) * np.random.default_rng(seed).standard_normal(n).astype(np.float32)
        out, loss, cap, (ms, rs, ns) = run_case(net, erb_t, mic, ref, near)
        name = f'case_{n}_{seed}'
        arrays = dict(mic=mic, ref=ref, near=near, out=out, loss=np.float32(loss))
        if cap:
            arrays.update(gru_in=cap['gru_in'][0].numpy(), gru_out=cap['gru_out'][0].numpy(),
                          mask=cap['mask'][0].numpy())
        if n <= 513:
            arrays.update(mic_spec=ms, ref_spec=rs, near_spec=ns, out_spec=cap['out_spec'][0].numpy())
        np.savez_compressed(os.path.join(HERE, name + '.npz'), **arrays)
        meta[name] = dict(n=n, seed=seed, double_talk=dt, out_len=int(out.shape[-1]), loss=loss)
        print(name, out.shape, loss)

    # 10 s utterance: summary only
    n, seed = 160000, 7
    mic, ref, near = synth.scene(n, seed)
    out, loss, _, _ = run_case(net, erb_t, mic, ref, near)
    h = hashlib.sha256(mic.tobytes() + ref.tobytes() + near.tobytes()).hexdigest()
    np.savez_compressed(os.path.join(HERE, 'long_160000_7.npz'), head=out[:2048], tail=out[-2048:],
                        rms=np.float64(np.sqrt(np.mean(out.astype(np.float64) ** 2))),
                        loss=np.float32(loss), out_len=np.int64(out.shape[-1]))
    meta['long_160000_7'] = dict(n=n, seed=seed, input_sha256=h, loss=loss)

    # ragged set: per-utterance (batch=1) outputs + the batched-call coupling hazard
    lens = [16077, 12345, 20000]
    per = {}
    mics, refs, nears = [], [], []
    for i, n in enumerate(lens):
        mic, ref, near = synth.scene(n, 100 + i)
        out, loss, _, _ = run_case(net, erb_t, mic, ref, near)
        per[f'out{i}'] = out
        per[f'loss{i}'] = np.float32(loss)
        mics.append(mic); refs.append(ref); nears.append(near)
    L = max(lens)
    pad = lambda xs: torch.tensor(np.stack([np.pad(x, (0, L - len(x))) for x in xs]))
    with torch.no_grad():
        bout, bloss = net(pad(mics), pad(refs), pad(nears), erb_t)
    diffs = [float(np.sqrt(np.mean((bout[i, :len(per[f'out{i}'])].numpy() - per[f'out{i}']) ** 2)))
             for i in range(3)]
    np.savez_compressed(os.path.join(HERE, 'ragged.npz'), lens=np.array(lens), **per)
    meta['ragged'] = dict(lens=lens, seeds=[100, 101, 102], batched_vs_single_rms=diffs)
    with open(os.path.join(HERE, 'golden_meta.json'), 'w') as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == '__main__':
    main()
