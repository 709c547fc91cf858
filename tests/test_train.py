"""Training step (scripts/train1.py:191-218).

CPU: the oracle's float64 backward + Adam against the reference's own
autograd / torch.optim.Adam (tests/golden/train.npz, made by
tests/golden/make_train_golden.py from /root/reference), the collate mirror.
GPU (`-m gpu`): aec_train_forward / aec_train_backward / aec_adam_step
through the C ABI against the golden and the oracle, and the reference's
training loop run unchanged on the drop-in (autograd + torch Adam)."""
import json
import os

import numpy as np
import pytest

import aec_oracle as O
from conftest import GOLDEN, PARAM_KEYS

LR = 1e-5                  # train_conf['lr'] (scripts/configs.py:12)
GRAD_RTOL = 2e-4           # relative L2 error per parameter tensor (f32 device vs f32 reference autograd)
LOSS_RTOL = 1e-5


@pytest.fixture(scope='module')
def tg():
    return dict(np.load(os.path.join(GOLDEN, 'train.npz')))


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))


def test_oracle_grads_match_reference_autograd(tg, golden_weights, golden_erb):
    erb = golden_erb.astype(np.float32)
    p = {k: golden_weights[k].astype(np.float64) for k in PARAM_KEYS}
    m = {k: np.zeros_like(p[k]) for k in PARAM_KEYS}
    v = {k: np.zeros_like(p[k]) for k in PARAM_KEYS}
    for it in range(2):
        loss, g = O.train_loss_and_grads(tg[f'mic{it}'], tg[f'ref{it}'], tg[f'near{it}'], erb, p)
        assert abs(loss - float(tg[f'loss{it}'])) <= LOSS_RTOL * abs(float(tg[f'loss{it}']))
        for k in PARAM_KEYS:
            assert _rel(g[k], tg[f'grad{it}/{k}']) <= 1e-5, (it, k)
        for k in PARAM_KEYS:
            p[k], m[k], v[k] = O.adam_step(p[k], g[k], m[k], v[k], it + 1, lr=LR)
            assert np.abs(p[k] - tg[f'param{it}/{k}']).max() <= 1e-7, (it, k)


def test_oracle_adam_matches_torch():
    import torch
    rng = np.random.default_rng(3)
    p0 = rng.standard_normal(257).astype(np.float32)
    t = torch.tensor(p0, requires_grad=True)
    opt = torch.optim.Adam([t], lr=1e-2, weight_decay=0.1)
    p, m, v = p0.astype(np.float64), np.zeros(257), np.zeros(257)
    for step in range(1, 4):
        g = rng.standard_normal(257).astype(np.float32)
        t.grad = torch.tensor(g)
        opt.step()
        p, m, v = O.adam_step(p, g.astype(np.float64), m, v, step, lr=1e-2, weight_decay=0.1)
        assert np.abs(p - t.detach().numpy()).max() <= 1e-6


def test_collate_pads_to_longest_nearend():
    import torch
    from aec_amd.train import TrainDataset
    items = [{k: np.full(n, i + 1, np.float32) for k in ('nearend_speech', 'nearend_mic', 'farend_speech', 'echo')}
             for i, n in enumerate([5, 9, 7])]
    items[1]['echo'] = np.ones(6, np.float32)            # shorter than its nearend_speech: padded too
    b = TrainDataset.collate_fn(items)
    assert b['n_samples'] == 9
    for k in ('nearend_speech', 'nearend_mic', 'farend_speech', 'echo'):
        assert b[k].shape == (3, 9) and b[k].dtype == torch.float32
    assert b['nearend_mic'][0].tolist() == [1.0] * 5 + [0.0] * 4
    assert b['echo'][1].tolist() == [1.0] * 6 + [0.0] * 3


def test_train_dataset_reads_h5lite_files(tmp_path):
    from aec_amd import h5lite
    from aec_amd.train import TrainDataset
    paths = []
    for i, n in enumerate([300, 700]):
        p = str(tmp_path / f'{i}.h5')
        h5lite.write_signals(p, {k: np.arange(n, dtype=np.float32) + j
                                 for j, k in enumerate(('nearend_speech', 'nearend_mic', 'farend_speech', 'echo'))})
        paths.append(p)
    ds = TrainDataset(paths)
    assert len(ds) == 2
    b = TrainDataset.collate_fn([ds[0], ds[1]])
    assert b['n_samples'] == 700
    assert np.array_equal(b['farend_speech'][0, :300].numpy(), np.arange(300, dtype=np.float32) + 2)
    assert not b['farend_speech'][0, 300:].any()


# ----------------------------------------------------------------------------- GPU
def _net(golden_weights, dev='cuda:0'):
    import torch
    import aec_amd
    from conftest import PARAM_KEYS as K
    net = aec_amd.Little_net(aec_amd.speech_conf, 32)
    sd = net.state_dict()
    for k in K:
        sd[k] = torch.from_numpy(golden_weights[k])
    net.load_state_dict(sd, strict=True)
    return net.to(dev).train()


def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    return torch


@pytest.mark.gpu
def test_train_forward_backward_vs_reference(tg, golden_weights, golden_erb):
    """aec_train_forward loss and aec_train_backward gradients of both golden
    iterations' batches (at the golden's own parameters) against the
    reference's autograd."""
    torch = _gpu()
    from aec_amd import _lib
    dev = 'cuda:0'
    h = _lib.Handle(0)
    h.set_erb(golden_erb.astype(np.float32))
    params = {k: golden_weights[k] for k in PARAM_KEYS}
    for it in range(2):
        blob = torch.from_numpy(np.concatenate([params[k].reshape(-1) for k in PARAM_KEYS]).astype(np.float32)).to(dev)
        mic, ref, near = (torch.from_numpy(tg[f'{s}{it}']).to(dev) for s in ('mic', 'ref', 'near'))
        B, N = mic.shape
        out = torch.empty(B, 256 * (N // 256), device=dev)
        loss = torch.empty((), device=dev)
        grad = torch.empty(blob.numel(), device=dev)
        st = torch.cuda.current_stream().cuda_stream
        h.set_weights_device(blob.data_ptr(), blob.numel(), st)
        h.train_forward(mic.data_ptr(), ref.data_ptr(), near.data_ptr(), N, B, N, out.data_ptr(), out.shape[1],
                        loss.data_ptr(), st)
        h.train_backward(None, grad.data_ptr(), st)
        torch.cuda.synchronize()
        assert abs(float(loss) - float(tg[f'loss{it}'])) <= 1e-5 * float(tg[f'loss{it}']), it
        assert np.abs(out[:, :1024].cpu().numpy() - tg[f'out_head{it}']).max() <= 1e-4
        g, o = grad.cpu().numpy(), 0
        for k in PARAM_KEYS:
            n = params[k].size
            assert _rel(g[o:o + n], tg[f'grad{it}/{k}'].reshape(-1)) <= GRAD_RTOL, (it, k)
            o += n
        params = {k: tg[f'param{it}/{k}'] for k in PARAM_KEYS}


@pytest.mark.gpu
def test_grad_loss_scales_and_backward_is_deterministic(tg, golden_weights, golden_erb):
    torch = _gpu()
    from aec_amd import _lib
    dev = 'cuda:0'
    h = _lib.Handle(0)
    h.set_erb(golden_erb.astype(np.float32))
    blob = torch.from_numpy(np.concatenate([golden_weights[k].reshape(-1) for k in PARAM_KEYS])).float().to(dev)
    mic, ref, near = (torch.from_numpy(tg[f'{s}0']).to(dev) for s in ('mic', 'ref', 'near'))
    B, N = mic.shape
    loss = torch.empty((), device=dev)
    st = torch.cuda.current_stream().cuda_stream
    h.set_weights_device(blob.data_ptr(), blob.numel(), st)
    h.train_forward(mic.data_ptr(), ref.data_ptr(), near.data_ptr(), N, B, N, None, 1, loss.data_ptr(), st)
    g1, g2, g3 = (torch.empty(blob.numel(), device=dev) for _ in range(3))
    two = torch.tensor(2.0, device=dev)
    h.train_backward(None, g1.data_ptr(), st)
    h.train_backward(None, g2.data_ptr(), st)
    h.train_backward(two.data_ptr(), g3.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(g1, g2)
    assert torch.allclose(g3, 2 * g1, rtol=1e-6, atol=0)


@pytest.mark.gpu
def test_native_adam_matches_oracle(golden_weights):
    torch = _gpu()
    from aec_amd import _lib
    dev = 'cuda:0'
    h = _lib.Handle(0)
    rng = np.random.default_rng(11)
    n = 12544 + 77
    p0 = rng.standard_normal(n).astype(np.float32)
    p, m, v = (torch.from_numpy(a).to(dev) for a in (p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)))
    pr, mr, vr = p0.astype(np.float64), np.zeros(n), np.zeros(n)
    st = torch.cuda.current_stream().cuda_stream
    for step in range(1, 5):
        g = (rng.standard_normal(n) * 10.0 ** rng.integers(-6, 1, n)).astype(np.float32)
        gt = torch.from_numpy(g).to(dev)
        h.adam_step(p.data_ptr(), gt.data_ptr(), m.data_ptr(), v.data_ptr(), n, step, 1e-3, 0.9, 0.999, 1e-8, 0.01, st)
        pr, mr, vr = O.adam_step(pr, g.astype(np.float64), mr, vr, step, lr=1e-3, weight_decay=0.01)
    torch.cuda.synchronize()
    assert np.abs(p.cpu().numpy() - pr).max() <= 2e-6
    # the multi-tensor launch (one param group): 3 tensors at different steps
    sizes = [12544, 77, 4096]
    ps = [torch.from_numpy(rng.standard_normal(s).astype(np.float32)).to(dev) for s in sizes]
    ms = [torch.zeros(s, device=dev) for s in sizes]
    vs = [torch.zeros(s, device=dev) for s in sizes]
    refs = [(t.cpu().numpy().astype(np.float64), np.zeros(s), np.zeros(s)) for t, s in zip(ps, sizes)]
    for step in range(1, 4):
        gs = [(rng.standard_normal(s) * 1e-3).astype(np.float32) for s in sizes]
        steps = [step, step + 1, step]
        gts = [torch.from_numpy(g).to(dev) for g in gs]          # kept alive across the async launch
        h.adam_step_multi([t.data_ptr() for t in ps], [t.data_ptr() for t in gts],
                          [t.data_ptr() for t in ms], [t.data_ptr() for t in vs], sizes, steps, 1e-3, 0.9, 0.999,
                          1e-8, 0.0, st)
        torch.cuda.synchronize()
        refs = [O.adam_step(pr_, g.astype(np.float64), mr_, vr_, s_, lr=1e-3)
                for (pr_, mr_, vr_), g, s_ in zip(refs, gs, steps)]
    for t, (pr_, _, _) in zip(ps, refs):
        assert np.abs(t.cpu().numpy() - pr_).max() <= 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize('optim', ['torch', 'native'])
def test_reference_training_loop_on_the_dropin(tg, golden_weights, golden_erb, optim):
    """train1.py:199-218 unchanged (net.train(), loss.backward(), Adam(lr).step())
    on the drop-in: two iterations reproduce the reference's parameters."""
    torch = _gpu()
    from aec_amd.train import Adam
    dev = 'cuda:0'
    net = _net(golden_weights, dev)
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    opt = (torch.optim.Adam if optim == 'torch' else Adam)([{'params': net.parameters()}], lr=LR, amsgrad=False)
    for it in range(2):
        mic, ref, near = (torch.from_numpy(tg[f'{s}{it}']).to(dev) for s in ('mic', 'ref', 'near'))
        opt.zero_grad()
        with torch.enable_grad():
            out, loss = net(mic, ref, near, erb_t)
        assert loss.requires_grad and loss.dim() == 0
        loss.backward()
        for k, p in net.named_parameters():
            assert _rel(p.grad.cpu().numpy(), tg[f'grad{it}/{k}']) <= GRAD_RTOL, (it, k)
        opt.step()
        for k, p in net.named_parameters():
            d_gpu = p.detach().cpu().numpy().astype(np.float64) - (golden_weights[k] if it == 0 else tg[f'param{it - 1}/{k}'])
            d_ref = tg[f'param{it}/{k}'].astype(np.float64) - (golden_weights[k] if it == 0 else tg[f'param{it - 1}/{k}'])
            # Adam's first steps move every entry by ~lr * sign(g): entries whose
            # gradient is ~0 in both may differ by up to 2 lr; all others agree
            bad = np.abs(d_gpu - d_ref) > 0.05 * LR + 1e-7
            assert bad.mean() <= 2e-3, (it, k, bad.sum())
            assert np.abs(p.detach().cpu().numpy() - tg[f'param{it}/{k}']).max() <= 2.05 * LR * (it + 1), (it, k)
            if it == 0:
                pass
        # keep the trajectories aligned: continue from the reference's parameters
        with torch.no_grad():
            for k, p in net.named_parameters():
                p.copy_(torch.from_numpy(tg[f'param{it}/{k}']))


@pytest.mark.gpu
def test_train_10s_batch16_vs_oracle(golden_weights, golden_erb):
    """train_conf batch size (16) at BASELINE C2 length (10 s, 626 BPTT steps):
    loss and gradients against the float64 oracle."""
    torch = _gpu()
    from aec_amd import synth
    dev = 'cuda:0'
    B, N = 16, 160000
    mic, ref, near = synth.batch(B, N, seed0=5100)
    net = _net(golden_weights, dev)
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    with torch.enable_grad():
        _, loss = net(*(torch.from_numpy(a).to(dev) for a in (mic, ref, near)), erb_t)
    loss.backward()
    ol, og = O.train_loss_and_grads(mic, ref, near, golden_erb.astype(np.float32), golden_weights)
    assert abs(float(loss.detach()) - ol) <= 1e-4 * ol
    for k, p in net.named_parameters():
        assert _rel(p.grad.cpu().numpy(), og[k]) <= 1e-3, k


@pytest.mark.gpu
def test_backward_of_stale_forward_raises(tg, golden_weights, golden_erb):
    torch = _gpu()
    dev = 'cuda:0'
    net = _net(golden_weights, dev)
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    mic, ref, near = (torch.from_numpy(tg[f'{s}1']).to(dev) for s in ('mic', 'ref', 'near'))
    with torch.enable_grad():
        _, l1 = net(mic, ref, near, erb_t)
        _, l2 = net(mic, ref, near, erb_t)
    with pytest.raises(RuntimeError, match='older forward'):
        l1.backward()
    l2.backward()
    assert all(p.grad is not None for p in net.parameters())
    with torch.enable_grad():
        out, l3 = net(mic, ref, near, erb_t)
    with pytest.raises(NotImplementedError):
        out.sum().backward()


def test_torch_train_port_matches_reference(tg, golden_weights, golden_erb):
    """The CPU baseline of the training figure (oracle/torch_port.py) follows
    the reference's autograd + Adam."""
    import torch
    from torch_port import TorchTrainPort
    port = TorchTrainPort(golden_weights, golden_erb.astype(np.float32), lr=LR)
    for it in range(2):
        loss = port.step(*(torch.from_numpy(tg[f'{s}{it}']) for s in ('mic', 'ref', 'near')))
        assert abs(loss - float(tg[f'loss{it}'])) <= 1e-5 * float(tg[f'loss{it}'])
        for k, p in zip(PARAM_KEYS, port.params):
            assert _rel(p.grad.numpy(), tg[f'grad{it}/{k}']) <= 1e-4, (it, k)


@pytest.mark.gpu
def test_chunked_scan_bptt_matches_serial(monkeypatch, golden_weights, golden_erb):
    """The chunked-scan BPTT (aec_train.hip T2a-c, used when T > 64) against
    the one-wave-per-stream serial recursion (AEC_BPTT_SERIAL=1) on ragged
    chunk counts (T = 157: a 13-step last chunk)."""
    torch = _gpu()
    from aec_amd import _lib, synth
    dev = 'cuda:0'
    B, N = 4, 40000
    mic, ref, near = (torch.from_numpy(a).to(dev) for a in synth.batch(B, N, seed0=8100))
    blob = torch.from_numpy(np.concatenate([golden_weights[k].reshape(-1) for k in PARAM_KEYS])).float().to(dev)
    grads = {}
    for serial in ('0', '1'):
        monkeypatch.setenv('AEC_BPTT_SERIAL', serial)
        h = _lib.Handle(0)
        h.set_erb(golden_erb.astype(np.float32))
        st = torch.cuda.current_stream().cuda_stream
        loss = torch.empty((), device=dev)
        g = torch.empty(blob.numel(), device=dev)
        h.set_weights_device(blob.data_ptr(), blob.numel(), st)
        h.train_forward(mic.data_ptr(), ref.data_ptr(), near.data_ptr(), N, B, N, None, 1, loss.data_ptr(), st)
        h.train_backward(None, g.data_ptr(), st)
        torch.cuda.synchronize()
        grads[serial] = g.cpu().numpy()
        del h
    o = 0
    for k in PARAM_KEYS:
        n = golden_weights[k].size
        assert _rel(grads['0'][o:o + n], grads['1'][o:o + n].astype(np.float64)) <= 1e-5, k
        o += n


@pytest.mark.gpu
def test_inference_call_invalidates_pending_backward(tg, golden_weights, golden_erb):
    """An inference forward on the same handle between the training forward
    and its backward overwrites the saved features: the backward must fail
    loudly, not return gradients of the wrong batch."""
    torch = _gpu()
    dev = 'cuda:0'
    net = _net(golden_weights, dev)
    erb_t = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    mic, ref, near = (torch.from_numpy(tg[f'{s}0']).to(dev) for s in ('mic', 'ref', 'near'))
    with torch.enable_grad():
        _, loss = net(mic, ref, near, erb_t)
    with torch.no_grad():
        net.eval()
        net(mic[:1], ref[:1], near[:1], erb_t)
        net.train()
    with pytest.raises(RuntimeError, match='older forward'):
        loss.backward()


def test_adam_state_dict_and_steplr_follow_torch():
    """train1.py:153-154 builds Adam + StepLR and checkpoints
    optimizer.state_dict() (train1.py:244-246): the native Adam keeps torch's
    param-group keys, accepts torch's state_dict and drives StepLR (CPU: no
    step taken)."""
    import torch
    from aec_amd.train import Adam
    p = [torch.nn.Parameter(torch.zeros(3)), torch.nn.Parameter(torch.zeros(2))]
    ref = torch.optim.Adam([{'params': p}], lr=LR, amsgrad=False)
    ours = Adam([{'params': p}], lr=LR, amsgrad=False)
    g_ref, g_ours = ref.state_dict()['param_groups'][0], ours.state_dict()['param_groups'][0]
    for k in ('lr', 'betas', 'eps', 'weight_decay', 'amsgrad', 'params'):
        assert g_ref[k] == g_ours[k], k
    ours.load_state_dict(ref.state_dict())
    sched = torch.optim.lr_scheduler.StepLR(ours, step_size=5, gamma=0.5)   # train_conf lr_decay_*
    for _ in range(5):
        sched.step()
    assert ours.param_groups[0]['lr'] == pytest.approx(LR * 0.5)
