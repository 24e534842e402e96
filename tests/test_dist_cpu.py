"""Multi-process plumbing of the sharded path on CPU (gloo, world_size 2).

The data path has no collective (independent matrices); what is
tested here is the setup broadcast of quant statistics, the round-robin
assignment and the max-over-ranks timing reduction -- the same code bench.py
runs over RCCL on a GPU node.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nf4_triton_dequantization_amd.sharding import (QuantStats, assign_round_robin, broadcast_quant_stats,
                                                    max_over_ranks, scatter_quant_stats)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stats(k):
    g = torch.Generator().manual_seed(7)
    out = []
    for i in range(k):
        m, n = 8 * (i + 1), 64 * (i + 2)
        nb = m * n // 64
        out.append(QuantStats(m, n, torch.randint(0, 256, (nb,), dtype=torch.uint8, generator=g),
                              torch.rand((nb + 255) // 256, generator=g),
                              [torch.float16, torch.bfloat16, torch.float32][i % 3]))
    return out


def _worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        src_stats = _stats(5) if rank == 0 else None
        got = broadcast_quant_stats(src_stats, torch.device("cpu"), src=0)
        ref = _stats(5)
        ok = len(got) == len(ref) and all(
            a.m == b.m and a.n == b.n and a.dtype == b.dtype and torch.equal(a.absmax, b.absmax)
            and torch.equal(a.absmax2, b.absmax2) for a, b in zip(got, ref))
        mine = assign_round_robin(5, world)[rank]
        slowest = max_over_ranks(float(rank + 1) * 1.5, torch.device("cpu"))
        empty = broadcast_quant_stats([] if rank == 0 else None, torch.device("cpu"), src=0)
        result_q.put((rank, ok, mine, slowest, len(empty)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_broadcast_and_assignment_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [True, True]
    assert res[0][2] == [0, 2, 4] and res[1][2] == [1, 3]
    assert res[0][3] == res[1][3] == 3.0
    assert res[0][4] == res[1][4] == 0


def test_round_robin_covers_everything():
    for items in (0, 1, 7, 8, 64):
        for world in (1, 2, 3, 8):
            parts = assign_round_robin(items, world)
            assert sorted(i for p in parts for i in p) == list(range(items))
            assert max(len(p) for p in parts) - min(len(p) for p in parts) <= 1
    with pytest.raises(ValueError):
        assign_round_robin(3, 0)


def _scatter_worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ref = _stats(7)
        owned = assign_round_robin(len(ref), world)
        per_rank = [[ref[i] for i in owned[r]] for r in range(world)] if rank == 0 else None
        got = scatter_quant_stats(per_rank, torch.device("cpu"), src=0)
        want = [ref[i] for i in owned[rank]]
        ok = len(got) == len(want) and all(
            a.m == b.m and a.n == b.n and a.dtype == b.dtype and torch.equal(a.absmax, b.absmax)
            and torch.equal(a.absmax2, b.absmax2) for a, b in zip(got, want))
        # a rank that owns nothing gets an empty list
        empty = scatter_quant_stats([[] for _ in range(world)] if rank == 0 else None, torch.device("cpu"), src=0)
        result_q.put((rank, ok, len(got), sum(int(s.absmax.numel()) for s in got), len(empty)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("world", [2, 3])
def test_scatter_sends_each_rank_only_its_own(world):
    """scatter_quant_stats: each rank receives exactly its round-robin share (uneven at
    world 3: 3/2/2 matrices), bit-equal, and nothing else."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    ref = _stats(7)
    owned = assign_round_robin(7, world)
    for r, ok, k, nbytes, nempty in res:
        assert ok and k == len(owned[r]) and nempty == 0
        assert nbytes == sum(int(ref[i].absmax.numel()) for i in owned[r])


def _subgroup_worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sub = dist.new_group([1, 2])  # every rank creates it; group rank 0 = global rank 1
        res = (rank, None, None)
        if rank in (1, 2):
            ref = _stats(5)
            owned = assign_round_robin(len(ref), 2)
            grank = dist.get_rank(sub)
            per_rank = [[ref[i] for i in owned[r]] for r in range(2)] if grank == 0 else None
            got = scatter_quant_stats(per_rank, torch.device("cpu"), src=0, group=sub)
            want = [ref[i] for i in owned[grank]]
            ok_s = len(got) == len(want) and all(
                torch.equal(a.absmax, b.absmax) and torch.equal(a.absmax2, b.absmax2) for a, b in zip(got, want))
            allb = broadcast_quant_stats(ref if grank == 0 else None, torch.device("cpu"), src=0, group=sub)
            ok_b = len(allb) == len(ref) and all(torch.equal(a.absmax, b.absmax) for a, b in zip(allb, ref))
            res = (rank, ok_s, ok_b)
        result_q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_scatter_and_broadcast_in_a_subgroup():
    """``src`` is a group rank: in a subgroup whose rank 0 is global rank 1, the scatter
    and the broadcast still start from that rank (dist.scatter takes the
    global rank)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_subgroup_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert res[0] == (0, None, None)
    assert res[1] == (1, True, True) and res[2] == (2, True, True)
