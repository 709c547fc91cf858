"""Training-step probe for rocprofv3 (run on the GPU box):
    python tools/train_probe.py --batch 16 --steps 10
prints bench.run_train's figure (one JSON line)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--batch', type=int, default=16)
ap.add_argument('--seconds', type=float, default=10.0)
ap.add_argument('--steps', type=int, default=10)
a = ap.parse_args()
import torch  # noqa: E402
print(json.dumps(bench.run_train(torch.device('cuda', 0), a.batch, int(a.seconds * 16000), a.steps)), flush=True)
