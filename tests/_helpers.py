"""Shared test helpers: golden-case loading, duck-typed modules, NaN-aware bit compare."""
from __future__ import annotations

import hashlib
import os
from types import SimpleNamespace

import numpy as np

import nf4_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

DT_CODE = {"f16": O.F16, "bf16": O.BF16, "f32": O.F32}


def torch_dtype(dt: str):
    import torch

    return {"f16": torch.float16, "bf16": torch.bfloat16, "f32": torch.float32}[dt]


def load_case(entry: dict) -> dict:
    with np.load(os.path.join(GOLDEN, entry["file"]), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def make_module(packed, absmax, a2, m, n, dt, device, *, a2_f16=None):
    """Duck-typed Linear4bit (only the attributes the reference reads)."""
    import torch

    a2_t = torch.from_numpy(a2_f16).to(device) if a2_f16 is not None else torch.from_numpy(a2).to(device)
    qs = SimpleNamespace(absmax=torch.from_numpy(absmax).to(device),
                         state2=SimpleNamespace(absmax=a2_t), dtype=torch_dtype(dt))
    w = SimpleNamespace(data=torch.from_numpy(packed).to(device).view(-1, 1), quant_state=qs)
    return SimpleNamespace(weight=w, out_features=m, in_features=n)


def out_bits(t) -> np.ndarray:
    """Raw output bits of a fp16/bf16/fp32 torch tensor as numpy uint16/uint32."""
    import torch

    t = t.detach().contiguous().cpu()
    if t.dtype == torch.float32:
        return t.view(torch.int32).numpy().view(np.uint32)
    return t.view(torch.int16).numpy().view(np.uint16)


def nan_mask(bits: np.ndarray, dt: str) -> np.ndarray:
    if dt == "f32":
        return np.isnan(bits.view(np.float32))
    if dt == "f16":
        return np.isnan(bits.view(np.float16))
    return np.isnan((bits.astype(np.uint32) << 16).view(np.float32))


def assert_bits_equal(got: np.ndarray, want: np.ndarray, dt: str, what: str = ""):
    """Bit-exact equality, except NaN payloads (torch itself emits 0x7FC0 or 0xFFFF)."""
    assert got.shape == want.shape, (got.shape, want.shape)
    gn, wn = nan_mask(got, dt), nan_mask(want, dt)
    assert np.array_equal(gn, wn), f"{what}: NaN positions differ"
    diff = (got != want) & ~gn
    if diff.any():
        idx = np.argwhere(diff)[:5]
        raise AssertionError(f"{what}: {int(diff.sum())} of {got.size} elements differ, first at "
                             f"{idx.tolist()}: got {got[tuple(idx[0])]:#x} want {want[tuple(idx[0])]:#x}")


def sha(bits: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(bits).tobytes()).hexdigest()


def max_abs_diff(got: np.ndarray, want: np.ndarray, dt: str) -> float:
    def f(b):
        if dt == "f16":
            return b.view(np.float16).astype(np.float64)
        if dt == "f32":
            return b.view(np.float32).astype(np.float64)
        return (b.astype(np.uint32) << 16).view(np.float32).astype(np.float64)

    a, b = f(got), f(want)
    ok = np.isfinite(a) & np.isfinite(b)
    return float(np.max(np.abs(a[ok] - b[ok]))) if ok.any() else 0.0


def big_samples(name: str):
    """(flat indices, expected bits) sampled from the reference output of a big golden case."""
    with np.load(os.path.join(GOLDEN, "big_samples.npz"), allow_pickle=False) as z:
        return z[name + "/idx"], z[name + "/bits"]


# ---- sentinel-guarded device buffers (the chunk-kernel and past-the-end suites) ----
GUARD = 64  # elements of sentinel before the output
# and after it: wide, because a wave past the end of the matrix once wrote its (empty)
# staged span at the element its unclamped row index pointed to, thousands of elements on
GUARD_AFTER = 1 << 18


def dev_bytes(a: np.ndarray, dev, offset=0):
    """`a` on the device at byte `offset` (0..3) into a fresh allocation, and that allocation."""
    import torch

    big = torch.zeros(a.size + 8, dtype=torch.uint8, device=dev)
    big[offset:offset + a.size] = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
    return big, big.data_ptr() + offset


def out_buffer(m, n, dt, dev, elem_offset):
    """An output of m*n elements at `elem_offset` elements into a sentinel-filled buffer."""
    import torch

    buf = torch.full((GUARD + elem_offset + m * n + GUARD_AFTER,), float("nan"), dtype=torch_dtype(dt), device=dev)
    bits = buf.view(torch.int32 if dt == "f32" else torch.int16)
    bits.fill_(0x5A5A5A5A if dt == "f32" else 0x5A5A)
    return buf, GUARD + elem_offset


def check_guarded(buf, start, m, n, dt, want, what):
    """The sentinels on both sides intact, and the output bit-equal to `want` ([m][n])."""
    import torch

    bits = buf.view(torch.int32 if dt == "f32" else torch.int16).cpu().numpy()
    sentinel = 0x5A5A5A5A if dt == "f32" else 0x5A5A
    assert (bits[:start] == sentinel).all(), f"{what}: write before the output"
    assert (bits[start + m * n:] == sentinel).all(), f"{what}: write past the output"
    got = bits[start:start + m * n].view(np.uint32 if dt == "f32" else np.uint16).reshape(m, n)
    assert_bits_equal(got, want, dt, what)
