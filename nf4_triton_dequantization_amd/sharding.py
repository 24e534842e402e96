"""Multi-GPU: independent NF4 weights sharded one-per-GPU, quant_state scattered over RCCL.

Scope (BASELINE.json config 5): dequantization has no exchange step
-- every weight matrix (and every row) is independent -- so ranks split the
matrices round-robin and never talk on the data path.  The only collective is
the distribution of the quantization statistics (``absmax`` u8 + nested
``state2.absmax`` fp32 + shape metadata) from the rank that loaded them, done
once at setup: ``scatter_quant_stats`` sends each rank only its own matrices'
statistics (per-destination point-to-point messages posted together, one xGMI
link each) -- what bench.py uses, by design instead of BASELINE's "RCCL broadcast
of quant_state": at C5 / N = 8 a rank receives 1 MiB + 16 KiB rather than all
8.5 MB; ``broadcast_quant_stats`` gives every rank everything (coalesced:
one u8 buffer, one fp32 buffer rather than one message per matrix).  ``src`` is a
rank of ``group`` in both (converted to the global rank the collectives take).  The packed 4-bit weights are resident on (or
loaded by) the rank that owns them and never cross the link.

One process per GPU, ``torch.distributed`` backend ``nccl`` (= RCCL on ROCm);
the same code runs on ``gloo`` with CPU tensors for the world_size-2 tests.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

_DT = {0: torch.float16, 1: torch.bfloat16, 2: torch.float32}
_DT_INV = {v: k for k, v in _DT.items()}


def assign_round_robin(num_items: int, world_size: int) -> List[List[int]]:
    """Item indices owned by each rank: item i goes to rank i % world_size."""
    if world_size <= 0:
        raise ValueError("world_size must be positive")
    return [list(range(r, num_items, world_size)) for r in range(world_size)]


@dataclass
class QuantStats:
    """Per-matrix statistics that travel: what ``nf4_dequant_ref`` needs besides the weight."""

    m: int
    n: int
    absmax: torch.Tensor    # uint8 [nb]
    absmax2: torch.Tensor   # fp32 [n2]
    dtype: torch.dtype


def broadcast_quant_stats(stats: Optional[Sequence[QuantStats]], device: torch.device, src: int = 0,
                          group=None) -> List[QuantStats]:
    """Broadcast every matrix's quant statistics from ``src`` to all ranks.

    ``stats`` is read on ``src`` only (ignored elsewhere).  Three collectives in
    total: a metadata header, the concatenated u8 absmax, the concatenated fp32
    nested absmax.  Returns the full list on every rank, on ``device``.
    """
    rank = dist.get_rank(group)
    gsrc = _global(src, group)  # collectives take the source's global rank
    if rank == src:
        if stats is None:
            raise ValueError("source rank must provide stats")
        meta, a1, a2 = _pack(list(stats), device)
        count = torch.tensor([meta.shape[0]], dtype=torch.int64, device=device)
    else:
        count = torch.zeros(1, dtype=torch.int64, device=device)
    dist.broadcast(count, gsrc, group=group)
    k = int(count.item())
    meta_d = meta.to(device) if rank == src else torch.zeros((k, 5), dtype=torch.int64, device=device)
    dist.broadcast(meta_d, gsrc, group=group)
    meta_h = meta_d.cpu()
    if rank != src:
        a1 = torch.empty(int(meta_h[:, 2].sum()) if k else 0, dtype=torch.uint8, device=device)
        a2 = torch.empty(int(meta_h[:, 3].sum()) if k else 0, dtype=torch.float32, device=device)
    if a1.numel():
        dist.broadcast(a1, gsrc, group=group)
    if a2.numel():
        dist.broadcast(a2, gsrc, group=group)
    return _unpack(meta_h, a1, a2)


def _global(r: int, group) -> int:
    """Global rank of group rank ``r`` (``src`` arguments here are group ranks)."""
    return r if group is None else dist.get_global_rank(group, r)


def _pack(stats: Sequence[QuantStats], device: torch.device):
    meta = torch.tensor([[s.m, s.n, s.absmax.numel(), s.absmax2.numel(), _DT_INV[s.dtype]] for s in stats],
                        dtype=torch.int64).reshape(-1, 5)
    a1 = torch.cat([s.absmax.reshape(-1).to(device) for s in stats]) if stats else \
        torch.zeros(0, dtype=torch.uint8, device=device)
    a2 = torch.cat([s.absmax2.reshape(-1).to(device, torch.float32) for s in stats]) if stats else \
        torch.zeros(0, dtype=torch.float32, device=device)
    return meta, a1, a2


def _unpack(meta_h: torch.Tensor, a1: torch.Tensor, a2: torch.Tensor) -> List[QuantStats]:
    out, o1, o2 = [], 0, 0
    for i in range(meta_h.shape[0]):
        m, n, nb, n2, dc = (int(v) for v in meta_h[i])
        out.append(QuantStats(m, n, a1[o1:o1 + nb], a2[o2:o2 + n2], _DT[dc]))
        o1 += nb
        o2 += n2
    return out


def scatter_quant_stats(per_rank: Optional[Sequence[Sequence[QuantStats]]], device: torch.device, src: int = 0,
                        group=None) -> List[QuantStats]:
    """Send each rank only the quant statistics of the matrices it owns.

    ``per_rank[r]`` (read on ``src`` only) lists rank r's matrices.  One
    fixed-size scatter of the per-rank sizes ([count, absmax bytes, nested
    absmax floats]), then, per destination, three point-to-point messages
    (metadata, the concatenated u8 absmax, the concatenated fp32 nested absmax)
    posted together, so on xGMI every peer's payload moves on its own link at
    once.  A rank receives what it uses and nothing else (at C5 / N = 8: 1 MiB
    + 16 KiB each, instead of every rank's 8 MiB).  Returns this rank's list,
    on ``device``.
    """
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if rank == src:
        if per_rank is None or len(per_rank) != world:
            raise ValueError("source rank must provide one stats list per rank")
        packed = [_pack(list(s), device) for s in per_rank]
        sizes = [torch.tensor([p[0].shape[0], p[1].numel(), p[2].numel()], dtype=torch.int64, device=device)
                 for p in packed]
    else:
        sizes = None
    mine_sz = torch.zeros(3, dtype=torch.int64, device=device)
    dist.scatter(mine_sz, sizes, src=_global(src, group), group=group)
    k, nb_tot, n2_tot = (int(v) for v in mine_sz.cpu())
    if rank == src:
        reqs = []
        for r in range(world):
            if r == src:
                continue
            meta, a1, a2 = packed[r]
            peer = _global(r, group)
            for t in (meta.to(device), a1, a2):
                if t.numel():
                    reqs.append(dist.isend(t.contiguous(), peer, group=group))
        for q in reqs:
            q.wait()
        meta, a1, a2 = packed[src]
        return _unpack(meta, a1, a2)
    meta_d = torch.zeros((k, 5), dtype=torch.int64, device=device)
    a1 = torch.empty(nb_tot, dtype=torch.uint8, device=device)
    a2 = torch.empty(n2_tot, dtype=torch.float32, device=device)
    peer = _global(src, group)
    reqs = [dist.irecv(t, peer, group=group) for t in (meta_d, a1, a2) if t.numel()]
    for q in reqs:
        q.wait()
    return _unpack(meta_d.cpu(), a1, a2)


def max_over_ranks(x: float, device: torch.device, group=None) -> float:
    """Max of a per-rank float over the group (bench timing: slowest rank decides)."""
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
