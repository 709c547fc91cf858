"""Multi-GPU sharding of utterances.

Utterances are independent: the normaliser, NLMS taps, GRU state and OLA
tail are all per stream. So one process per GPU processes its own shard and
no data crosses GPUs during compute. The only collectives are scalar ones
outside the data path:
- `max_over_ranks` for the bench clock;
- `sum_over_ranks` for run-level metric sums (frames, Σmic², Σout²).

Both use the process group's backend: RCCL ("nccl") on the GPU box, gloo in
the CPU tests.
"""
from __future__ import annotations

import heapq
from typing import List, Sequence

import torch
import torch.distributed as dist


def frames_of(n: int) -> int:
    """Work of one utterance in frames, T = N//256 + 1 (attention_ccrn.py:48-49)."""
    return int(n) // 256 + 1


def balanced_shards(lengths: Sequence[int], world: int) -> List[List[int]]:
    """Greedy longest-first assignment of utterance indices to `world` ranks.

    Each utterance, longest first, goes to the rank with the least total
    frames so far. Ties are broken by the lower index, then the lower rank, so
    every rank computes the same table with no broadcast. Each shard's
    indices are returned in ascending order. The makespan is at most the ideal
    share plus one utterance (LPT bound).
    """
    if world < 1:
        raise ValueError('world must be >= 1')
    order = sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i))
    heap = [(0, r) for r in range(world)]
    shards: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        shards[r].append(i)
        heapq.heappush(heap, (load + frames_of(lengths[i]), r))
    return [sorted(s) for s in shards]


def _dev():
    if dist.get_backend() == 'nccl':
        return torch.device('cuda', torch.cuda.current_device())
    return torch.device('cpu')


def max_over_ranks(x: float) -> float:
    """Max of a per-rank scalar (the bench's elapsed time); identity when not distributed."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_dev())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values: Sequence[float]) -> List[float]:
    """Elementwise sum of per-rank metric vectors; identity when not distributed."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=_dev())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]
