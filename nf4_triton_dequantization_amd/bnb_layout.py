"""bitsandbytes ``Linear4bit`` / ``Params4bit`` / ``QuantState`` layout stand-in + NF4 quantizer.

bitsandbytes is not installed here, yet the drop-in boundary is
defined by its layout: the reference reads ``module.weight.data``
(uint8 ``[numel/2, 1]``), ``weight.quant_state.absmax`` (uint8),
``quant_state.state2.absmax`` (fp32), ``quant_state.dtype`` and
``module.out_features / in_features``; its harness additionally asserts the
fields checked by ``assert_correct_bnb`` (reference benchmark.py:18-28):
``quant_state.code`` fp32, ``offset`` fp32, ``blocksize == 64``,
``state2.code`` fp32, ``state2.blocksize == 256``.

This module supplies objects with exactly that layout, plus the producer side
(SURVEY §8f row 3): ``quantize_nf4`` restates bitsandbytes' published NF4
quantizer (blockwise absmax, nearest NF4 code, high nibble first) and its
nested 8-bit "dynamic map" compression of the absmax (``compress_statistics``).
Being a restatement of an absent library, its bit-level agreement with real
bitsandbytes is unpinned; what the tests pin is the layout and that the
``semantics="bnb"`` dequant inverts it.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn

# NF4 code points (the same 16 fp32 values as kernel_optimized.py:234-239).
NF4_CODE = torch.tensor(
    [-1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
     -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
     0.07958029955625534, 0.16093020141124725, 0.24611230194568634, 0.33791524171829224,
     0.44070982933044434, 0.5626170039176941, 0.7229568362236023, 1.0], dtype=torch.float32)


def dynamic_map(signed: bool = True, max_exponent_bits: int = 7, total_bits: int = 8) -> torch.Tensor:
    """The 256-entry dynamic (exponent + linear fraction) code book bitsandbytes uses
    for the nested absmax.  Each decade 10^(e-6), e = 0..6, contributes the
    midpoints of a linear partition of [0.1, 1]; then 0 and 1 are added, the
    list is padded with zeros to 256 and sorted."""
    vals = []
    frac_bits = total_bits - 1 - max_exponent_bits
    for e in range(max_exponent_bits):
        count = 2 ** (e + frac_bits) + 1 if signed else 2 ** (e + frac_bits + 1) + 1
        edges = torch.linspace(0.1, 1.0, count, dtype=torch.float32)
        mids = (edges[:-1] + edges[1:]) / 2.0
        scale = 10.0 ** (-(max_exponent_bits - 1) + e)
        vals += (scale * mids).tolist()
        if signed:
            vals += (-scale * mids).tolist()
    extra = 2 ** frac_bits - 1
    if extra > 0:
        edges = torch.linspace(0.1, 1.0, extra + 1, dtype=torch.float32)
        mids = (edges[:-1] + edges[1:]) / 2.0
        scale = 10.0 ** (-(max_exponent_bits - 1) + max_exponent_bits - 1)
        vals += (scale * mids).tolist()
        if signed:
            vals += (-scale * mids).tolist()
    vals += [0.0, 1.0]
    vals += [0.0] * (2 ** total_bits - len(vals))
    vals.sort()
    return torch.tensor(vals, dtype=torch.float32)


class QuantState:
    """Field layout of ``bitsandbytes.functional.QuantState`` (what the boundary reads)."""

    def __init__(self, absmax, shape=None, code=None, blocksize=None, quant_type=None, dtype=None,
                 offset=None, state2: Optional["QuantState"] = None):
        self.absmax = absmax
        self.shape = shape
        self.code = code
        self.blocksize = blocksize
        self.quant_type = quant_type
        self.dtype = dtype
        self.offset = offset
        self.state2 = state2
        self.nested = state2 is not None

    def to(self, device):
        self.absmax = self.absmax.to(device)
        if self.code is not None:
            self.code = self.code.to(device)
        if self.offset is not None:
            self.offset = self.offset.to(device)
        if self.state2 is not None:
            self.state2.to(device)
        return self


def _nearest_code(x: torch.Tensor, code: torch.Tensor) -> torch.Tensor:
    """Index of the nearest entry of a sorted code book (ties to the lower index)."""
    mids = (code[1:] + code[:-1]) / 2.0
    return torch.bucketize(x, mids, right=False)


def quantize_blockwise_8bit(a: torch.Tensor, code: torch.Tensor, blocksize: int = 256):
    """Blockwise absmax 8-bit quantization of a flat fp32 vector with a code book."""
    n = a.numel()
    nblk = (n + blocksize - 1) // blocksize
    pad = nblk * blocksize - n
    ap = torch.nn.functional.pad(a.reshape(-1), (0, pad)).view(nblk, blocksize)
    amax = ap.abs().amax(dim=1).clamp_min(torch.finfo(torch.float32).tiny)
    q = _nearest_code((ap / amax[:, None]).reshape(-1), code.to(a.device))[:n]
    return q.to(torch.uint8), amax.to(torch.float32)


def quantize_nf4(w: torch.Tensor, blocksize: int = 64, compress_statistics: bool = True,
                 blocksize2: int = 256, quant_storage=torch.uint8):
    """NF4-quantize ``w`` ([out, in] float) into the bitsandbytes Params4bit layout.

    Returns ``(packed uint8 [numel/2, 1], QuantState)``.  ``quant_state.dtype`` is
    ``w.dtype``.
    """
    shape = w.shape
    dev = w.device
    flat = w.detach().reshape(-1).to(torch.float32)
    n = flat.numel()
    if n % 2:
        flat = torch.nn.functional.pad(flat, (0, 1))
    nblk = (n + blocksize - 1) // blocksize
    pad = nblk * blocksize - flat.numel()
    blocks = torch.nn.functional.pad(flat, (0, pad)).view(nblk, blocksize)
    absmax = blocks.abs().amax(dim=1).to(torch.float32)
    safe = torch.where(absmax > 0, absmax, torch.ones_like(absmax))
    idx = _nearest_code((blocks / safe[:, None]).reshape(-1), NF4_CODE.to(dev))[: flat.numel()]
    idx = idx.to(torch.uint8)
    packed = ((idx[0::2] << 4) | idx[1::2]).to(torch.uint8).view(-1, 1)
    if quant_storage != torch.uint8:
        packed = packed.view(quant_storage)
    code = NF4_CODE.to(dev)
    if compress_statistics:
        offset = absmax.mean()
        c2 = dynamic_map(signed=True).to(dev)
        qabs, abs2 = quantize_blockwise_8bit(absmax - offset, c2, blocksize2)
        state2 = QuantState(absmax=abs2, code=c2, blocksize=blocksize2, quant_type=None, dtype=torch.float32)
        qs = QuantState(absmax=qabs, shape=shape, code=code, blocksize=blocksize, quant_type="nf4",
                        dtype=w.dtype, offset=offset.reshape(()), state2=state2)
    else:
        qs = QuantState(absmax=absmax, shape=shape, code=code, blocksize=blocksize, quant_type="nf4",
                        dtype=w.dtype)
    return packed, qs


class Params4bit(nn.Parameter):
    """uint8 packed NF4 storage with an attached ``quant_state`` (bnb ``Params4bit`` layout)."""

    def __new__(cls, data: torch.Tensor, quant_state: Optional[QuantState] = None):
        self = super().__new__(cls, data, requires_grad=False)
        self.quant_state = quant_state
        return self

    def to(self, *args, **kwargs):
        moved = super().to(*args, **kwargs)
        out = Params4bit(moved.data, self.quant_state)
        if self.quant_state is not None:
            dev = moved.device
            self.quant_state.to(dev)
        return out


class Linear4bit(nn.Module):
    """Minimal ``bitsandbytes.nn.Linear4bit`` stand-in (NF4, optional nested absmax).

    ``Linear4bit(in_features, out_features, bias=None, compute_dtype=..., compress_statistics=True,
    quant_type="nf4")`` quantizes a kaiming-uniform fp32 weight at construction (bnb
    quantizes on ``.to("cuda")``; the resulting layout is the same).  ``forward`` uses
    bitsandbytes semantics through the HIP kernel.
    """

    def __init__(self, input_features: int, output_features: int, bias=None, compute_dtype=None,
                 compress_statistics: bool = True, quant_type: str = "nf4", device=None,
                 weight: Optional[torch.Tensor] = None, blocksize: int = 64):
        super().__init__()
        if quant_type != "nf4":
            raise ValueError("only quant_type='nf4' is supported")
        self.in_features = input_features
        self.out_features = output_features
        self.compute_dtype = compute_dtype
        if weight is None:
            weight = torch.empty(output_features, input_features, dtype=torch.float32, device=device)
            nn.init.kaiming_uniform_(weight, a=math.sqrt(5))
        packed, qs = quantize_nf4(weight.to(torch.float32), blocksize=blocksize,
                                  compress_statistics=compress_statistics)
        qs.dtype = compute_dtype if compute_dtype is not None else weight.dtype
        qs.shape = torch.Size((output_features, input_features))
        self.weight = Params4bit(packed, qs)
        self.bias = None if not bias else nn.Parameter(torch.zeros(output_features, device=device))

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        if self.weight.quant_state is not None:
            self.weight.quant_state.to(self.weight.device)
        return self

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from .kernel import dequantize_nf4_bnb

        w = dequantize_nf4_bnb(self)
        y = x.to(w.dtype) @ w.t()
        if self.bias is not None:
            y = y + self.bias.to(y.dtype)
        return y
