"""Multi-GPU sharding of utterances.

Utterances are independent: the normaliser, NLMS taps, GRU state and OLA
tail are all per stream. So one process per GPU processes its own shard and
no data crosses GPUs during compute. The collectives sit outside the data
path:
- `max_over_ranks` for the bench clock;
- `sum_over_ranks` for run-level metric sums (frames, Σmic², Σout²);
- `gather_to_root`: the end-of-run gather of enhanced waveforms to rank 0
  (north_star: RCCL over xGMI only gathers the enhanced waveforms), used by
  the CLI's ``--gather`` mode.

Both use the process group's backend: RCCL ("nccl") on the GPU box, gloo in
the CPU tests.
"""
from __future__ import annotations

import heapq
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
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


_BOUND: Optional[int] = None     # this rank's GPU, set by bind_device()


def local_rank() -> int:
    """This process's GPU index under torchrun (LOCAL_RANK), 0 otherwise."""
    return int(os.environ.get('LOCAL_RANK', '0'))


def bind_device(local: Optional[int] = None) -> int:
    """Make GPU `local` (default LOCAL_RANK) this rank's current device and the
    device of every collective below.  RCCL needs one GPU per rank: a rank
    left on cuda:0 duplicates rank 0's GPU and the first collective fails or
    hangs."""
    global _BOUND
    local = local_rank() if local is None else int(local)
    torch.cuda.set_device(local)
    _BOUND = local
    return local


def init_process_group(backend: Optional[str] = None) -> None:
    """Join the torchrun process group, one GPU per rank: bind LOCAL_RANK's GPU
    first and hand it to RCCL as the group's device (`device_id`), as
    bench.py does; gloo (CPU) when no GPU is visible."""
    if dist.is_initialized():
        return
    if backend is None:
        backend = 'nccl' if torch.cuda.is_available() else 'gloo'
    if backend == 'nccl':
        local = bind_device()
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        dist.init_process_group(backend)


def _dev():
    """Device of the collectives: the rank's bound GPU under RCCL, CPU under gloo."""
    if dist.get_backend() == 'nccl':
        return torch.device('cuda', _BOUND if _BOUND is not None else local_rank())
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


def gather_to_root(outputs: Dict[int, np.ndarray], root: int = 0) -> Optional[Dict[int, np.ndarray]]:
    """Gather every rank's {utterance index: float32 waveform} to `root`.

    Two collectives on the process group's device (RCCL over xGMI on the GPU
    box, gloo in the CPU tests): an all_gather of the per-rank sample counts,
    then one gather of each rank's waveforms packed into a flat float32 buffer
    (padded to the largest rank) with an int64 (index, length) table.
    Returns the merged dict on `root`, None elsewhere; identity when not
    distributed."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return dict(outputs)
    dev = _dev()
    world, rank = dist.get_world_size(), dist.get_rank()
    keys = sorted(outputs)
    table = np.array([[k, len(outputs[k])] for k in keys], np.int64).reshape(-1, 2)
    counts = torch.tensor([len(keys), int(table[:, 1].sum()) if len(keys) else 0], dtype=torch.int64, device=dev)
    allc = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(allc, counts)
    allc = [c.tolist() for c in allc]
    max_utt = max(1, max(c[0] for c in allc))
    max_smp = max(1, max(c[1] for c in allc))
    tab = torch.full((max_utt, 2), -1, dtype=torch.int64)
    tab[:len(keys)] = torch.from_numpy(table)
    flat = torch.zeros(max_smp, dtype=torch.float32)
    if keys:
        flat[:int(table[:, 1].sum())] = torch.from_numpy(np.concatenate([np.asarray(outputs[k], np.float32)
                                                                          for k in keys]))
    tab, flat = tab.to(dev), flat.to(dev)
    tabs = [torch.empty_like(tab) for _ in range(world)] if rank == root else None
    flats = [torch.empty_like(flat) for _ in range(world)] if rank == root else None
    dist.gather(tab, tabs, dst=root)
    dist.gather(flat, flats, dst=root)
    if rank != root:
        return None
    merged: Dict[int, np.ndarray] = {}
    for r in range(world):
        t = tabs[r].cpu().numpy()
        f = flats[r].cpu().numpy()
        off = 0
        for k, n in t[:allc[r][0]]:
            merged[int(k)] = f[off:off + int(n)].copy()
            off += int(n)
    return merged
