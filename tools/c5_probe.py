"""C5 per-hop step probe for rocprofv3 (GPU box): python tools/c5_probe.py [--dtype fp8] [--hops 200]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--dtype', default='fp8')
ap.add_argument('--hops', type=int, default=200)
a = ap.parse_args()
print(json.dumps(bench.run_c5_stream(torch.device('cuda', 0), hops=a.hops, dtype=a.dtype)), flush=True)
