"""GPU: the fused per-hop streaming step (include/aec_hip.h aec_stream_*)
reproduces the batch path (aec_process) hop by hop.

The streaming kernel runs the batch kernels' own arithmetic (aec_frame.h
helpers; the GRU step restates gru_kernel's accumulation order), so the bar
is BIT-EXACT equality with the batch output (observed on MI355X: max abs
difference 0 for the post-filter and the 4-tap NLMS path), integer framing
exact (step k emits output hop k-1).

The normaliser x - mean(x)/std(x) (ERB.py:254-256) needs the whole
utterance, so the streamed hops are normalised here with the same float64
statistic the batch path uses, rounded to float32, zero past the end.
"""
import numpy as np
import pytest
import torch

from conftest import PARAM_KEYS

pytestmark = pytest.mark.gpu

NLMS = dict(taps=4, mu=0.3, beta=0.5, delta=1e-4)      # aec_amd.configs.nlms_conf


def _net(golden_weights, nlms):
    import aec_amd
    net = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=nlms).eval()
    sd = net.state_dict()
    for k in PARAM_KEYS:
        sd[k] = torch.from_numpy(golden_weights[k])
    net.load_state_dict(sd, strict=True)
    return net.to('cuda:0')


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-30))


def _normalised(x):
    c = np.float32(np.mean(x, dtype=np.float64) / np.std(x.astype(np.float64), ddof=1))
    return (x - c).astype(np.float32)


def _scenes(lens, seed0):
    from aec_amd import synth
    return [synth.scene(n, seed0 + i) for i, n in enumerate(lens)]


@pytest.mark.parametrize('nlms', [None, NLMS, dict(NLMS, taps=1), dict(NLMS, taps=8)],
                         ids=['postfilter', 'nlms4', 'nlms1', 'nlms8'])
def test_stream_equals_batch(golden_weights, golden_erb, nlms):
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    net = _net(golden_weights, nlms)
    dev = 'cuda:0'
    erb = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    lens = [4097, 2125, 9000, 256]
    sc = _scenes(lens, 500)
    L = max(lens)
    pad = lambda k: torch.tensor(np.stack([np.pad(s[k], (0, L - len(s[k]))) for s in sc]), device=dev)
    with torch.no_grad():
        ref_out, _ = net.forward_ragged(pad(0), pad(1), None, erb, lens)
    torch.cuda.synchronize()
    nh = L // 256 + 1                                      # hops fed: 0 .. L//256
    B = len(lens)
    mic = np.zeros((B, 256 * nh), np.float32)
    far = np.zeros_like(mic)
    for b, s in enumerate(sc):
        mic[b, :lens[b]] = _normalised(s[0])
        far[b, :lens[b]] = _normalised(s[1])
    mic_d, far_d = torch.tensor(mic, device=dev), torch.tensor(far, device=dev)
    with torch.no_grad():
        net.stream_open(B, erb)
        outs = [net.stream_step(mic_d[:, 256 * k:256 * (k + 1)], far_d[:, 256 * k:256 * (k + 1)])
                for k in range(nh)]
    torch.cuda.synchronize()
    got = torch.cat(outs[1:], dim=1).cpu().numpy()        # step k emits hop k-1
    ref_np = ref_out.cpu().numpy()
    for b, n in enumerate(lens):
        no = 256 * (n // 256)
        r = _rel(got[b, :no], ref_np[b, :no])
        print(f'stream {b} n={n}: rel {r:.2e} max abs {float(np.abs(got[b, :no] - ref_np[b, :no]).max()):.2e}')
        assert np.array_equal(got[b, :no], ref_np[b, :no]), (b, n, r)

    # per-stream reset: stream 3 restarts with utterance 0 (the others keep going on zeros)
    with torch.no_grad():
        net.stream_reset(3)
        mic2 = torch.zeros_like(mic_d)
        far2 = torch.zeros_like(far_d)
        mic2[3], far2[3] = mic_d[0], far_d[0]
        outs = [net.stream_step(mic2[:, 256 * k:256 * (k + 1)], far2[:, 256 * k:256 * (k + 1)])[3]
                for k in range(nh)]
    torch.cuda.synchronize()
    got3 = torch.cat(outs[1:]).cpu().numpy()
    no = 256 * (lens[0] // 256)
    assert np.array_equal(got3[:no], ref_np[0, :no])


def test_stream_argument_errors(golden_weights, golden_erb):
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    net = _net(golden_weights, None)
    dev = 'cuda:0'
    with pytest.raises(RuntimeError):
        net.stream_step(torch.zeros(2, 256, device=dev), torch.zeros(2, 256, device=dev))
    net.stream_open(2, torch.tensor(golden_erb, dtype=torch.float32, device=dev))
    with pytest.raises(ValueError):
        net.stream_step(torch.zeros(3, 256, device=dev), torch.zeros(3, 256, device=dev))
    with pytest.raises(RuntimeError):
        net.stream_reset(5)


def test_stream_single_stream_strided_hops(golden_weights, golden_erb):
    """B = 1 with hops taken from a wider buffer at an odd row stride (ld_in =
    257 floats): the kernel reads rows at any stride; output bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    net = _net(golden_weights, NLMS)
    dev = 'cuda:0'
    erb = torch.tensor(golden_erb, dtype=torch.float32, device=dev)
    n = 5000
    (s,) = _scenes([n], 900)
    with torch.no_grad():
        ref_out, _ = net.forward_ragged(torch.tensor(s[0], device=dev)[None], torch.tensor(s[1], device=dev)[None],
                                        None, erb, [n])
    nh = n // 256 + 1
    mic = np.zeros(256 * nh, np.float32)
    far = np.zeros_like(mic)
    mic[:n], far[:n] = _normalised(s[0]), _normalised(s[1])
    buf = torch.zeros(2, nh, 257, device=dev)              # row stride 257: odd, not 16-B aligned
    buf[0, :, :256] = torch.tensor(mic.reshape(nh, 256), device=dev)
    buf[1, :, :256] = torch.tensor(far.reshape(nh, 256), device=dev)
    with torch.no_grad():
        net.stream_open(1, erb)
        outs = [net.stream_step(buf[0, k:k + 1, :256], buf[1, k:k + 1, :256]) for k in range(nh)]
    torch.cuda.synchronize()
    got = torch.cat(outs[1:], dim=1)[0].cpu().numpy()
    no = 256 * (n // 256)
    assert np.array_equal(got[:no], ref_out[0, :no].cpu().numpy())
