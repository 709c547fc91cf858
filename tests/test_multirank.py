"""N > 1 path on CPU: world-size-2 gloo process groups.

The HIP path has no data-path collective: every rank runs its own streams.
What must be right by construction is:
- the shard table: every rank derives the same one, shards are disjoint and
  complete, and the load is balanced;
- the scalar reductions the bench and the run metrics use.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aec_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, lengths, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        mine = shard.balanced_shards(lengths, world)[rank]
        tables = [None] * world
        dist.all_gather_object(tables, mine)
        el = shard.max_over_ranks(1.0 + rank)
        sums = shard.sum_over_ranks([sum(shard.frames_of(lengths[i]) for i in mine), 1.0])
        q.put((rank, tables, el, sums))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_gloo_shards_and_reductions(world):
    lengths = [160000, 64123, 191999, 100000, 75000, 160000, 255, 513, 120000, 99999, 64000]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, lengths, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    tables = res[0][1]
    assert all(r[1] == tables for r in res)                           # same table on every rank
    flat = sorted(i for t in tables for i in t)
    assert flat == list(range(len(lengths)))                          # disjoint and complete
    for _, _, el, sums in res:
        assert el == float(world)                                     # max over ranks of 1 + rank
        assert sums[0] == sum(shard.frames_of(n) for n in lengths)
        assert sums[1] == float(world)


def _gather_worker(rank, world, port, lengths, q):
    import numpy as np
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        mine = shard.balanced_shards(lengths, world)[rank]
        outs = {k: (np.arange(256 * (lengths[k] // 256), dtype=np.float32) * 1e-3 + k) for k in mine}
        got = shard.gather_to_root(outs)
        q.put((rank, None if got is None else {k: v.tolist() for k, v in got.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_gloo_gather_to_root(world):
    # 3 ranks over 2 utterances: one rank has nothing to send
    import numpy as np
    lengths = [1000, 70000] if world == 3 else [1000, 70000, 255, 9000, 513]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, lengths, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] is None for r in res[1:])
    got = res[0][1]
    assert sorted(got) == list(range(len(lengths)))
    for k, n in enumerate(lengths):
        exp = np.arange(256 * (n // 256), dtype=np.float32) * 1e-3 + k
        assert np.array_equal(np.asarray(got[k], np.float32), exp)


def test_balanced_shards_properties():
    import random
    rng = random.Random(0)
    for world in [1, 2, 4, 8]:
        lengths = [rng.randint(64000, 192000) for _ in range(257)]
        sh = shard.balanced_shards(lengths, world)
        assert sorted(i for s in sh for i in s) == list(range(len(lengths)))
        loads = [sum(shard.frames_of(lengths[i]) for i in s) for s in sh]
        ideal = sum(loads) / world
        assert max(loads) <= ideal + max(shard.frames_of(n) for n in lengths)   # LPT bound
    assert shard.balanced_shards([], 4) == [[], [], [], []]
    assert shard.balanced_shards([5, 5, 5], 8)[3:] == [[]] * 5
    with pytest.raises(ValueError):
        shard.balanced_shards([1], 0)


def test_rank_binds_its_local_gpu_for_rccl(monkeypatch):
    """Under torchrun every rank must run its collectives on ITS GPU
    (LOCAL_RANK), not on cuda:0: the CLI's group init binds the device first
    and hands it to RCCL, and the collectives' device follows (shard._dev).
    torch.cuda / the process group are stubbed: no GPU here."""
    from aec_amd import tester
    calls = {}
    monkeypatch.setenv('WORLD_SIZE', '2')
    monkeypatch.setenv('RANK', '1')
    monkeypatch.setenv('LOCAL_RANK', '1')
    monkeypatch.setattr(shard, '_BOUND', None)
    monkeypatch.setattr(torch.cuda, 'is_available', lambda: True)
    monkeypatch.setattr(torch.cuda, 'set_device', lambda d: calls.setdefault('set_device', int(d)))
    monkeypatch.setattr(torch.cuda, 'current_device', lambda: 0)   # what an unbound rank would see
    state = {'init': False}

    def fake_init(backend, **kw):
        calls['backend'] = backend
        calls['device_id'] = kw.get('device_id')
        state['init'] = True

    monkeypatch.setattr(dist, 'is_initialized', lambda: state['init'])
    monkeypatch.setattr(dist, 'is_available', lambda: True)
    monkeypatch.setattr(dist, 'init_process_group', fake_init)
    monkeypatch.setattr(dist, 'get_rank', lambda: 1)
    monkeypatch.setattr(dist, 'get_world_size', lambda: 2)
    monkeypatch.setattr(dist, 'get_backend', lambda *a: 'nccl')
    assert tester._dist() == (1, 2)
    assert calls['set_device'] == 1
    assert calls['backend'] == 'nccl' and calls['device_id'] == torch.device('cuda', 1)
    assert shard._dev() == torch.device('cuda', 1)
    # the device a collective tensor is built on: the bound GPU even with cuda:0 current
    monkeypatch.setattr(shard, '_BOUND', None)
    assert shard._dev() == torch.device('cuda', 1)              # LOCAL_RANK when not bound yet
