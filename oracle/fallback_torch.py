"""Torch-CPU restatement of the reference fallback's EXECUTION SHAPE -- TEST/BENCH INFRASTRUCTURE ONLY.

The reference's CPU path is ``_aggressive_pytorch_t4``
(/root/reference/nf4_triton_dequantization/kernel_optimized.py:208-314).  It
cannot travel to the GPU box, so ``bench.py`` times this restatement there as
the "reference fallback" CPU figure ("CPU-baseline plan", row 1).
What makes the fallback slow is its structure, so that structure is kept:

* wrap/truncate of the quant statistics by ``repeat`` (:245-261);
* one fp32 scale column per 64-block, computed in a Python loop over blocks
  (:263-270);
* whole-matrix nibble extraction into int64 index tensors and two LUT gathers
  producing fp32 ``[m, n/2]`` temporaries (:281-287);
* a Python loop over blocks, and inside it one strided column write (with the
  cast to the output dtype) per output column (:289-312).

Same arithmetic as ``nf4_oracle`` (fp32 ``q / 127``, fp32 multiply by the
nested scale, fp32 product with the code, one RNE cast), pinned against
``tests/golden/`` by ``tests/test_oracle_golden.py``.  Only ``tests/`` and
``bench.py``'s ``cpu_baseline`` leg import it; the product never does.
"""
from __future__ import annotations

import torch

# kernel_optimized.py:234-239, the same fp32 values as nf4_oracle.NF4_BITS
_CODES = (
    -1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
    -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
    0.07958029955625534, 0.16093020141124725, 0.24611230194568634, 0.33791524171829224,
    0.44070982933044434, 0.5626170039176941, 0.7229568362236023, 1.0,
)


def _fit(v: torch.Tensor, count: int) -> torch.Tensor:
    """First `count` entries of v repeated end to end (the reference's wrap, :247-251)."""
    if v.numel() >= count:
        return v[:count]
    times = -(-count // v.numel())
    return v.repeat(times)[:count]


def block_scales(a1: torch.Tensor, a2: torch.Tensor, m: int, n: int) -> torch.Tensor:
    """fp32 [m, blocks] scales, one block column per loop trip (:240-270)."""
    nblk = -(-n // 64)
    ngrp = -(-nblk // 4)
    q = _fit(a1.reshape(-1), m * nblk).reshape(m, nblk)
    nested = _fit(a2.reshape(-1), m * ngrp).reshape(m, ngrp).to(torch.float32)
    out = torch.zeros((m, nblk), dtype=torch.float32)
    for b in range(nblk):
        out[:, b] = (q[:, b].to(torch.float32) / 127.0) * nested[:, b // 4]
    return out


def dequant_fallback(packed: torch.Tensor, absmax: torch.Tensor, absmax2, m: int, n: int,
                     dtype: torch.dtype) -> torch.Tensor:
    """[m, n] `dtype` tensor: double dequant when absmax is uint8, else the single-quant branch."""
    if packed.dtype != torch.uint8:
        packed = packed.to(torch.uint8)
    rows = packed.contiguous().view(m, -1)
    nblk = -(-n // 64)
    if absmax.dtype == torch.uint8:
        scales = block_scales(absmax, absmax2, m, n)
    else:
        scales = absmax.reshape(m, -1)[:, :nblk].to(torch.float32)
    lut = torch.tensor(_CODES, dtype=torch.float32)
    lo_idx = (rows & 0xF).long()
    hi_idx = ((rows >> 4) & 0xF).long()
    lo_val = lut[lo_idx]
    hi_val = lut[hi_idx]
    out = torch.empty((m, n), dtype=dtype)
    for b in range(nblk):
        c0 = 64 * b
        c1 = min(c0 + 64, n)
        s = scales[:, b:b + 1]
        p0, p1 = c0 // 2, (c1 + 1) // 2
        hi_blk = hi_val[:, p0:p1] * s
        lo_blk = lo_val[:, p0:p1] * s
        for j in range(p1 - p0):
            col = c0 + 2 * j
            if col < n:
                out[:, col] = hi_blk[:, j].to(dtype)      # high nibble -> even column
            if col + 1 < n:
                out[:, col + 1] = lo_blk[:, j].to(dtype)  # low nibble -> odd column
    return out
