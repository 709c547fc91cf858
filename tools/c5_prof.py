#!/usr/bin/env python3
"""C5 per-hop step under a tracer: bench.run_c5_stream (256 streams, hipGraph NLMS -> DCCRN fp8)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.argv = ['bench.py']
import bench  # noqa: E402
import torch  # noqa: E402

r = bench.run_c5_stream(torch.device('cuda', 0), B=int(os.environ.get('STREAMS', '256')), hops=int(os.environ.get('HOPS', '200')), sweep=())
print(json.dumps(r))
