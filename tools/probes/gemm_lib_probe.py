"""Round 6: the C3 LSTM input projection (M = 2 B T = 320,512, N = 8,192, K = 1,024 bf16, + bias)
through hipBLASLt (torch.nn.functional.linear), and the copy that would materialise its implicit
A rows (each row = 4 bins x 256 channels at the level-6 map's row stride) as a contiguous matrix."""
import time
import torch

dev = 'cuda:0'
M, N, K = 320512, 8192, 1024
F = M // 2
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.03
b = torch.randn(N, device=dev, dtype=torch.bfloat16)
# implicit-A source as cat[L] of net_conf: [F][4 bins][2 * 512 ch] (encoder half at 512..1023 = (s, q))
cat = torch.randn(F, 4, 1024, device=dev, dtype=torch.bfloat16)


def gather():
    # row (f, s): bins d = 0..3, channels 512 + 256 s + q
    return cat[:, :, 512:].reshape(F, 4, 2, 256).permute(0, 2, 1, 3).reshape(M, K)


for name, fn in [('hipblaslt linear+bias', lambda: torch.nn.functional.linear(x, w, b)),
                 ('gather copy (implicit A -> contiguous)', lambda: gather().contiguous()),
                 ('gather + linear+bias', lambda: torch.nn.functional.linear(gather(), w, b))]:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    print(name, f'{dt * 1e3:.3f} ms', f'{2 * M * N * K / dt / 1e12:.0f} TFLOP/s', flush=True)
