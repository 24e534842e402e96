"""Synthetic workloads of the BASELINE.json configs: the deterministic input
generator and the shape sets, shared by bench.py, tools/, tests/ and the
fixture script (oracle/gen_golden.py).

Not the product and not the oracle: the product (``nf4_triton_dequantization_amd``)
takes caller tensors and never generates data; the oracle (``oracle/``) only
checks.  The generator is a stateless splitmix64 counter hash so the GPU box
regenerates bit-identical inputs without depending on torch's RNG version.

Configs (BASELINE.json ``configs``):

* C1 1024x1024 NF4->fp16 (CPU plumbing case)
* C2 4096x4096 NF4->bf16 (the headline)
* C3 Llama-3-8B linear weights, 32 layers x {q,o 4096x4096; k,v 1024x4096;
  gate,up 14336x4096; down 4096x14336}; C3b the "4096/11008" set BASELINE names
  (Llama-2-7B: q,k,v,o 4096x4096; gate,up 11008x4096; down 4096x11008)
* C4 4096x4096 fp16 vs bf16 (output-dtype sweep)
* C5 8192x8192 NF4->bf16, one matrix per GPU (8 matrices over 8 GPUs)
"""
from __future__ import annotations

import numpy as np

LLAMA3_8B = [(4096, 4096), (1024, 4096), (1024, 4096), (4096, 4096), (14336, 4096), (14336, 4096), (4096, 14336)]
LLAMA2_7B = [(4096, 4096)] * 4 + [(11008, 4096), (11008, 4096), (4096, 11008)]
LLAMA_LAYERS = 32
C5_SHAPE = (8192, 8192)
C5_MATRICES = 8


def c3_shapes(variant: str = "llama3", layers: int = LLAMA_LAYERS):
    """Every weight of one pass, in model order: [(m, n), ...] (224 for 32 layers)."""
    per_layer = {"llama3": LLAMA3_8B, "llama2": LLAMA2_7B}[variant]
    return [s for _ in range(layers) for s in per_layer]


def algorithmic_bytes(m: int, n: int, out_bytes: int, nb: int | None = None, n2: int | None = None) -> int:
    """N/2 packed + N*s output + nb absmax bytes + 4*min(n2, m*G) unique nested absmax.

    nb / n2 default to real bitsandbytes counts (ceil(N/64), ceil(nb/256)).
    """
    N = m * n
    if nb is None:
        nb = (N + 63) // 64
    if n2 is None:
        n2 = (nb + 255) // 256
    groups = ((n + 63) // 64 + 3) // 4
    return N // 2 + N * out_bytes + nb + 4 * min(n2, m * groups)


# ----------------------------------------------------------------------------
# deterministic inputs (splitmix64 counter hash)
# ----------------------------------------------------------------------------
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed: int, count: int, stream: int = 0) -> np.ndarray:
    """``count`` splitmix64 outputs for (seed, stream): a stateless counter hash."""
    with np.errstate(over="ignore"):
        base = np.uint64((seed * 0x100000001B3 + stream * 0x5851F42D4C957F2D) & 0xFFFFFFFFFFFFFFFF)
        x = base + (np.arange(1, count + 1, dtype=np.uint64) * _GOLDEN)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def splitmix64_bytes(seed: int, nbytes: int, stream: int = 0) -> np.ndarray:
    words = splitmix64(seed, (nbytes + 7) // 8, stream)
    return words.view(np.uint8)[:nbytes].copy()


def uniform_f32(seed: int, count: int, lo: float, hi: float, stream: int = 0) -> np.ndarray:
    """Uniform fp32 in [lo, hi) from the top 24 bits of splitmix64."""
    u = (splitmix64(seed, count, stream) >> np.uint64(40)).astype(np.float64) / float(1 << 24)
    return (lo + (hi - lo) * u).astype(np.float32)


def normal_f32(seed: int, count: int, stream: int = 0) -> np.ndarray:
    """Box-Muller N(0,1) in fp32 (includes negatives)."""
    w = splitmix64(seed, count, stream)
    u1 = ((w >> np.uint64(40)).astype(np.float64) + 0.5) / float(1 << 24)
    u2 = ((w & np.uint64(0xFFFFFF)).astype(np.float64) + 0.5) / float(1 << 24)
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)).astype(np.float32)


def make_inputs(m: int, n: int, seed: int, *, nb: int | None = None, n2: int | None = None,
                a2_kind: str = "uniform"):
    """Synthetic bnb-layout inputs: packed bytes, A1 u8, A2 fp32.

    Default counts are real-bnb counts: nb = ceil(m*n/64), n2 = ceil(nb/256).
    """
    numel = m * n
    if nb is None:
        nb = (numel + 63) // 64
    if n2 is None:
        n2 = (nb + 255) // 256
    packed = splitmix64_bytes(seed, numel // 2, stream=1)
    a1 = splitmix64_bytes(seed, nb, stream=2)
    if a2_kind == "uniform":
        a2 = uniform_f32(seed, n2, 1e-3, 1e-2, stream=3)
    elif a2_kind == "normal":
        a2 = normal_f32(seed, n2, stream=3)
    else:
        raise ValueError(a2_kind)
    return packed, a1, a2
