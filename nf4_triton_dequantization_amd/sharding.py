"""Multi-GPU: independent NF4 weights sharded one-per-GPU, quant_state broadcast over RCCL.

Scope (BASELINE.json config 5): dequantization has no exchange step
-- every weight matrix (and every row) is independent -- so ranks split the
matrices round-robin and never talk on the data path.  The only collective is
the broadcast of the quantization statistics (``absmax`` u8 + nested
``state2.absmax`` fp32 + shape metadata) from the rank that loaded them, done
once at setup as two coalesced broadcasts (one u8 buffer, one fp32 buffer)
rather than one message per matrix: on xGMI a ~1 MiB message is latency-bound,
so fewer, larger messages win.  The packed 4-bit weights are resident on (or
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
    if rank == src:
        if stats is None:
            raise ValueError("source rank must provide stats")
        meta = torch.tensor([[s.m, s.n, s.absmax.numel(), s.absmax2.numel(), _DT_INV[s.dtype]] for s in stats],
                            dtype=torch.int64).reshape(-1, 5)
        count = torch.tensor([meta.shape[0]], dtype=torch.int64, device=device)
    else:
        count = torch.zeros(1, dtype=torch.int64, device=device)
    dist.broadcast(count, src, group=group)
    k = int(count.item())
    if rank == src:
        meta_d = meta.to(device)
    else:
        meta_d = torch.zeros((k, 5), dtype=torch.int64, device=device)
    dist.broadcast(meta_d, src, group=group)
    meta_h = meta_d.cpu()
    nb_tot = int(meta_h[:, 2].sum()) if k else 0
    n2_tot = int(meta_h[:, 3].sum()) if k else 0
    if rank == src:
        a1 = torch.cat([s.absmax.reshape(-1).to(device) for s in stats]) if k else \
            torch.zeros(0, dtype=torch.uint8, device=device)
        a2 = torch.cat([s.absmax2.reshape(-1).to(device, torch.float32) for s in stats]) if k else \
            torch.zeros(0, dtype=torch.float32, device=device)
    else:
        a1 = torch.empty(nb_tot, dtype=torch.uint8, device=device)
        a2 = torch.empty(n2_tot, dtype=torch.float32, device=device)
    if nb_tot:
        dist.broadcast(a1, src, group=group)
    if n2_tot:
        dist.broadcast(a2, src, group=group)
    out, o1, o2 = [], 0, 0
    for i in range(k):
        m, n, nb, n2, dc = (int(v) for v in meta_h[i])
        out.append(QuantStats(m, n, a1[o1:o1 + nb], a2[o2:o2 + n2], _DT[dc]))
        o1 += nb
        o2 += n2
    return out


def max_over_ranks(x: float, device: torch.device, group=None) -> float:
    """Max of a per-rank float over the group (bench timing: slowest rank decides)."""
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
