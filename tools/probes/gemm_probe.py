"""Time the LSTM input projection shape (M = 2 B T = 320,512, N = 8192,
K = 1024, bf16) through torch (hipBLASLt / rocBLAS) for comparison with the
hand-written row GEMM (~6.2 ms per layer)."""
import time
import torch

dev = 'cuda:0'
M, N, K = 320512, 8192, 1024
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.03
b = torch.randn(N, device=dev, dtype=torch.bfloat16)
for name, fn in [('linear+bias', lambda: torch.nn.functional.linear(x, w, b)),
                 ('matmul', lambda: x @ w.t())]:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    print(name, f'{dt * 1e3:.3f} ms', f'{2 * M * N * K / dt / 1e12:.0f} TFLOP/s', flush=True)
