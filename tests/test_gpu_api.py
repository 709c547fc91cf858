"""GPU tests of the C-ABI's call semantics (include/aec_hip.h) rather than of
its arithmetic: concurrency of handles on different streams, the work-list
cache, and the weight-version bookkeeping of the native Adam.

* Two handles on two HIP streams with ragged lengths that change on every
  call: no call synchronises the device (prepare_lists uploads its work lists
  in stream order from pinned staging), so the two streams' work overlaps in
  time (HIP events bracket every call) and every output equals the same
  call made alone, bit for bit.
* The work-list cache keys on the lengths AND on whether near is given (the
  near slot of the per-signal lengths depends on it).
* aec_amd.train.Adam bumps the parameters' version counters, so an eval
  forward after the step uploads the new weights.
"""
import numpy as np
import pytest
import torch

from conftest import PARAM_KEYS

pytestmark = pytest.mark.gpu


def _net(golden_weights, nlms=None):
    import aec_amd
    net = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=nlms).eval()
    sd = net.state_dict()
    for k in PARAM_KEYS:
        sd[k] = torch.from_numpy(golden_weights[k])
    net.load_state_dict(sd, strict=True)
    return net.to('cuda:0')


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')


def test_two_handles_two_streams_overlap(golden_weights, golden_erb):
    _need_gpu()
    dev = torch.device('cuda:0')
    erb = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    nets = [_net(golden_weights), _net(golden_weights)]          # one handle each
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    B, L = 16, 320000              # 20 s streams: ~0.4 ms of GPU work per call, above the host's issue time
    g = torch.Generator(device=dev).manual_seed(12)
    sig = [[0.1 * torch.randn(B, L, device=dev, generator=g) for _ in range(3)] for _ in range(2)]
    rng = np.random.default_rng(5)
    shapes = [[rng.integers(L // 2, L + 1, B).tolist() for _ in range(2)] for _ in range(6)]
    with torch.no_grad():
        for k in range(2):                                          # size the workspaces (grow-only)
            nets[k].forward_ragged(*sig[k], erb, [L] * B)
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t0.record(torch.cuda.current_stream(dev))
        torch.cuda.synchronize()
        for s in streams:
            s.wait_stream(torch.cuda.current_stream(dev))
        ev, outs = [], []
        for lens in shapes:                                         # new ragged lengths every call
            pair = []
            for k in range(2):
                with torch.cuda.stream(streams[k]):
                    a = torch.cuda.Event(enable_timing=True)
                    b = torch.cuda.Event(enable_timing=True)
                    a.record(streams[k])
                    o, l = nets[k].forward_ragged(*sig[k], erb, lens[k])
                    b.record(streams[k])
                    pair.append((a, b, o, l))
            ev.append(pair)
        torch.cuda.synchronize()
        spans = [[(t0.elapsed_time(a), t0.elapsed_time(b)) for a, b, _, _ in pair] for pair in ev]
        overlaps = sum(1 for (a0, a1), (b0, b1) in spans if b0 < a1 and a0 < b1)
        assert overlaps >= len(shapes) // 2, spans
        # every result equals the same call made alone on the default stream
        for lens, pair in zip(shapes, ev):
            for k in range(2):
                o1, l1 = nets[k].forward_ragged(*sig[k], erb, lens[k])
                assert torch.equal(pair[k][2], o1), k
                assert torch.equal(pair[k][3], l1), k


def test_list_cache_keys_on_near(golden_weights, golden_erb):
    """Same lengths, first without near (the near slot of the lists takes the
    mic length), then with a shorter near of the same frame count: the second
    call must rebuild the lists and match a fresh handle."""
    _need_gpu()
    dev = torch.device('cuda:0')
    erb = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    from aec_amd import synth
    n = 16250                                    # 63 hops; the shorter signals keep the frame count
    mic, ref, near = (torch.from_numpy(a).to(dev) for a in synth.batch(2, n, seed0=77))
    l3 = np.array([[n, n, n - 110], [n, n - 100, n - 120]], np.int64)
    net = _net(golden_weights)
    with torch.no_grad():
        net.forward_ragged(mic, ref, None, erb, l3)
        o, l = net.forward_ragged(mic, ref, near, erb, l3)
        o2, l2 = _net(golden_weights).forward_ragged(mic, ref, near, erb, l3)
    torch.cuda.synchronize()
    assert torch.equal(o, o2)
    # row 0's near is silent over its stored length: the reference's loss is 0/0 = NaN there
    assert np.array_equal(l.cpu().numpy(), l2.cpu().numpy(), equal_nan=True)


def test_native_adam_step_reaches_eval_forward(golden_weights, golden_erb):
    """train forward + backward, an eval forward (uploads and caches the weight
    key), Adam.step(), another eval forward: the last one runs on the updated
    weights (equal to a fresh module loaded with them)."""
    _need_gpu()
    import aec_amd
    from aec_amd.train import Adam
    dev = torch.device('cuda:0')
    erb = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    from aec_amd import synth
    mic, ref, near = (torch.from_numpy(a).to(dev) for a in synth.batch(2, 16000, seed0=88))
    net = _net(golden_weights).train()
    opt = Adam(net.parameters(), lr=1e-2)
    opt.zero_grad()
    _, loss = net(mic, ref, near, erb)
    loss.backward()
    net.eval()
    with torch.no_grad():
        before, _ = net(mic, ref, near, erb)
    opt.step()
    with torch.no_grad():
        after, _ = net(mic, ref, near, erb)
        fresh = aec_amd.Little_net(aec_amd.speech_conf, 32).eval()
        fresh.load_state_dict({k: v.detach().cpu() for k, v in net.state_dict().items()})
        want, _ = fresh.to(dev)(mic, ref, near, erb)
    torch.cuda.synchronize()
    assert not torch.equal(before, after)
    assert torch.equal(after, want)
