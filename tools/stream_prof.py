#!/usr/bin/env python3
"""Phase timing (s_memtime cycles, block 0) of the fused per-hop kernels of
crn_stream.hip from a -DAEC_STREAM_PROF build (tools/build_variant.sh sprof
tree -DAEC_STREAM_PROF; AEC_HIP_LIB=.../ab/sprof.so): C5's 256-stream fp8 step."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
import aec_amd  # noqa: E402
from aec_amd import _lib  # noqa: E402

dev = torch.device('cuda', 0)
torch.manual_seed(0)
net = aec_amd.dccrn2.DCCRN(dict(aec_amd.net_conf), dtype='fp8', nlms=aec_amd.nlms_conf).eval().to(dev)
B = 256
net.stream_open(B, device=dev)
mic = 0.1 * torch.randn(B, 256, device=dev)
far = 0.1 * torch.randn(B, 256, device=dev)
out = torch.empty(B, 256, device=dev)
lib = _lib.load()
acc = []
with torch.no_grad():
    for k in range(60):
        net.stream_step(mic, far, out)
        torch.cuda.synchronize()
        if k >= 10:
            buf = np.zeros((2, 16), np.uint64)
            assert lib.aec_debug_stream_prof(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
            acc.append(buf.astype(np.int64))
a = np.median(np.stack(acc), axis=0)
names = {0: ['start', 'loads', 'fft', 'nlms+x0', 'enc0', 'enc1', 'enc2'],
         1: ['start', 'loads', 'dec cl3', 'dec cl2', 'mask level', 'mask apply', 'irfft', 'store']}
for kern in (0, 1):
    nm = names[kern]
    row = a[kern]
    print(['enc', 'dec'][kern], 'total', row[len(nm) - 1] - row[0], 'cycles')
    for i in range(1, len(nm)):
        print(f'   {nm[i]:12s} {row[i] - row[i - 1]:8.0f}')
