"""CPU oracle for NF4 double-dequantization -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  The product (``nf4_triton_dequantization_amd``)
never imports it; it fails loudly when its HIP library is missing.

Two independent restatements of the reference algorithm live here:

* ``dequant_ref_np`` / ``dequant_single_np`` / ``dequant_bnb_np`` -- vectorised
  numpy, written from the semantics in SURVEY.md §0.1;
* ``COracle`` -- ctypes binding of ``oracle/nf4_oracle.c`` (built by
  ``oracle/Makefile`` into ``oracle/_build/libnf4oracle.so``).

Both are pinned against ``tests/golden/`` (fixtures produced by running the
reference fallback ``_aggressive_pytorch_t4``,
/root/reference/nf4_triton_dequantization/kernel_optimized.py:208-314, via
``oracle/gen_golden.py``).

The deterministic input generator (``splitmix64_bytes`` & co.) lives in
``workloads.py`` at the repo root and is re-exported here.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

F16 = 0
BF16 = 1
F32 = 2

# kernel_optimized.py:234-239 (fp32 bit patterns of the decimal constants).
NF4_BITS = np.array(
    [0xBF800000, 0xBF3239B1, 0xBF066B30, 0xBECA32A0, 0xBE91A24D, 0xBE3D353F,
     0xBDBA7871, 0x00000000, 0x3DA2FAFF, 0x3E24CAE3, 0x3E7C04DD, 0x3EAD033A,
     0x3EE1A4B8, 0x3F1007AB, 0x3F3913B3, 0x3F800000], dtype=np.uint32)
NF4_LUT = NF4_BITS.view(np.float32)

_HERE = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------
# deterministic inputs: the shared generator lives in /workloads.py (the bench and
# tools use it too); re-exported here for the fixture script and the tests
# ----------------------------------------------------------------------------
import sys as _sys  # noqa: E402

_REPO = os.path.dirname(_HERE)
if _REPO not in _sys.path:
    _sys.path.insert(0, _REPO)
from workloads import make_inputs, normal_f32, splitmix64, splitmix64_bytes, uniform_f32  # noqa: E402,F401


def golden_case_inputs(m: int, n: int, seed: int, ov: dict):
    """Inputs of one tests/golden case (shared by oracle/gen_golden.py and the tests).

    ``ov`` keys: stride (packed bytes per row), nb, n2, a2_kind ("uniform" |
    "normal"), a2_scale, single (extra absmax columns -> fp32 single-quant absmax).
    """
    stride = ov.get("stride", n // 2)
    nb = ov.get("nb", (m * n + 63) // 64)
    n2 = ov.get("n2", (nb + 255) // 256)
    packed = splitmix64_bytes(seed, m * stride, stream=1)
    a1 = splitmix64_bytes(seed, nb, stream=2)
    if ov.get("a2_kind", "uniform") == "normal":
        a2 = normal_f32(seed, n2, stream=3)
    else:
        a2 = uniform_f32(seed, n2, 1e-3, 1e-2, stream=3)
    if "a2_scale" in ov:
        a2 = (a2 * np.float32(ov["a2_scale"] / 1e-2)).astype(np.float32)
    absmax_single = None
    if "single" in ov:
        bpr = (n + 63) // 64
        absmax_single = uniform_f32(seed, m * (bpr + ov["single"]), 1e-3, 1.0, stream=4)
    return packed, a1, a2, absmax_single


# ----------------------------------------------------------------------------
# rounding
# ----------------------------------------------------------------------------
def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)).astype(np.uint16)
    nan = np.isnan(x)
    if nan.any():
        r = np.where(nan, np.uint16(0x7FC0), r)
    return r


def f32_to_f16_bits(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        return np.ascontiguousarray(x, dtype=np.float32).astype(np.float16).view(np.uint16)


def to_bits(x: np.ndarray, dtype: int) -> np.ndarray:
    """Output bits: uint16 for fp16/bf16 (RNE), uint32 for fp32 (unrounded)."""
    if dtype == F32:
        return np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    return f32_to_bf16_bits(x) if dtype == BF16 else f32_to_f16_bits(x)


def out_bits_dtype(dtype: int):
    return np.uint32 if dtype == F32 else np.uint16


# ----------------------------------------------------------------------------
# numpy restatement
# ----------------------------------------------------------------------------
def _decode(packed: np.ndarray, m: int, n: int):
    if packed.size % m:
        raise ValueError("packed weight cannot be viewed as (m, -1)")
    stride = packed.size // m
    if stride < (n + 1) // 2:
        raise ValueError("packed rows shorter than ceil(n/2)")
    rows = packed.reshape(m, stride)[:, : (n + 1) // 2]
    nib = np.empty((m, 2 * rows.shape[1]), dtype=np.uint8)
    nib[:, 0::2] = rows >> 4          # high nibble -> even column (:108-110)
    nib[:, 1::2] = rows & 0xF         # low nibble  -> odd column
    return NF4_LUT[nib[:, :n]]


def ref_scales(a1: np.ndarray, a2: np.ndarray, m: int, n: int) -> np.ndarray:
    """fp32 [m, bpr] scales, reference double-dequant (:40-45, :246-270)."""
    bpr = (n + 63) // 64
    g = (bpr + 3) // 4
    r = np.arange(m, dtype=np.int64)[:, None]
    b = np.arange(bpr, dtype=np.int64)[None, :]
    q = a1[(r * bpr + b) % a1.size].astype(np.float32)
    s1 = q / np.float32(127.0)
    return (s1 * a2.astype(np.float32)[(r * g + b // 4) % a2.size]).astype(np.float32)


def _apply(vals: np.ndarray, scales: np.ndarray, n: int, dtype: int) -> np.ndarray:
    s = np.repeat(scales, 64, axis=1)[:, :n]
    return to_bits((vals * s).astype(np.float32), dtype)


def dequant_ref_np(packed, a1, a2, m, n, dtype):
    """uint16 bits [m, n] of the reference double-dequant output."""
    if a1.size == 0 or a2.size == 0:
        raise ValueError("empty absmax")
    return _apply(_decode(packed, m, n), ref_scales(a1, a2, m, n), n, dtype)


def dequant_single_np(packed, absmax, m, n, dtype):
    """Reference single-quant branch (:273-274): absmax fp32 viewable as (m, -1)."""
    bpr = (n + 63) // 64
    if absmax.size % m:
        raise ValueError("absmax cannot be viewed as (m, -1)")
    sc = absmax.astype(np.float32).reshape(m, -1)
    if sc.shape[1] < bpr:
        raise ValueError("absmax rows shorter than blocks per row")
    return _apply(_decode(packed, m, n), sc[:, :bpr], n, dtype)


def dequant_bnb_np(packed, a1, code2, a2, offset, numel, dtype, blocksize=64, blocksize2=256):
    """bitsandbytes semantics on the flat stream (parity unpinned)."""
    nblk = (numel + blocksize - 1) // blocksize
    blk = np.arange(nblk)
    am = (code2.astype(np.float32)[a1[:nblk]] * a2.astype(np.float32)[blk // blocksize2]).astype(np.float32)
    am = (am + np.float32(offset)).astype(np.float32)
    nib = np.empty(2 * packed.size, dtype=np.uint8)
    nib[0::2] = packed >> 4
    nib[1::2] = packed & 0xF
    vals = NF4_LUT[nib[:numel]]
    s = np.repeat(am, blocksize)[:numel]
    return to_bits((vals * s).astype(np.float32), dtype)


# ----------------------------------------------------------------------------
# C restatement (ctypes)
# ----------------------------------------------------------------------------
_LIB_PATH = os.path.join(_HERE, "_build", "libnf4oracle.so")


def build_c_oracle(quiet: bool = True) -> str:
    """Compile oracle/nf4_oracle.c (make); returns the .so path."""
    subprocess.run(["make", "-C", _HERE, "-s"], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)
    return _LIB_PATH


class COracle:
    """ctypes wrapper over the C restatement (single-threaded, scalar)."""

    def __init__(self, path: str | None = None):
        path = path or _LIB_PATH
        if not os.path.exists(path):
            build_c_oracle()
        self.lib = ctypes.CDLL(path)
        i64, p = ctypes.c_int64, ctypes.c_void_p
        L = self.lib
        L.nf4o_dequant_ref.argtypes = [p, i64, p, i64, p, i64, p, ctypes.c_int, i64, i64]
        L.nf4o_set_threads.argtypes = [ctypes.c_int]
        L.nf4o_set_threads.restype = None
        L.nf4o_dequant_single.argtypes = [p, i64, p, i64, p, ctypes.c_int, i64, i64]
        L.nf4o_dequant_bnb.argtypes = [p, p, i64, p, p, i64, ctypes.c_float, p, ctypes.c_int, i64, i64, i64]
        L.nf4o_dequant_bnb_single.argtypes = [p, p, i64, p, ctypes.c_int, i64, i64]
        for f in (L.nf4o_dequant_ref, L.nf4o_dequant_single, L.nf4o_dequant_bnb, L.nf4o_dequant_bnb_single):
            f.restype = ctypes.c_int
        L.nf4o_f32_to_bf16.argtypes = [ctypes.c_float]
        L.nf4o_f32_to_bf16.restype = ctypes.c_uint16
        L.nf4o_f32_to_f16.argtypes = [ctypes.c_float]
        L.nf4o_f32_to_f16.restype = ctypes.c_uint16

    @staticmethod
    def _p(a):
        return a.ctypes.data_as(ctypes.c_void_p)

    def set_threads(self, t: int) -> None:
        """OpenMP threads for the row loop (CPU-baseline timing; results do not depend on it)."""
        self.lib.nf4o_set_threads(int(t))

    def dequant_ref(self, packed, a1, a2, m, n, dtype):
        packed = np.ascontiguousarray(packed, np.uint8)
        a1 = np.ascontiguousarray(a1, np.uint8)
        a2 = np.ascontiguousarray(a2, np.float32)
        out = np.empty((m, n), dtype=out_bits_dtype(dtype))
        rc = self.lib.nf4o_dequant_ref(self._p(packed), packed.size, self._p(a1), a1.size,
                                       self._p(a2), a2.size, self._p(out), dtype, m, n)
        if rc:
            raise ValueError("nf4o_dequant_ref rejected the shapes")
        return out

    def dequant_single(self, packed, absmax, m, n, dtype):
        packed = np.ascontiguousarray(packed, np.uint8)
        absmax = np.ascontiguousarray(absmax, np.float32)
        out = np.empty((m, n), dtype=out_bits_dtype(dtype))
        rc = self.lib.nf4o_dequant_single(self._p(packed), packed.size, self._p(absmax), absmax.size,
                                          self._p(out), dtype, m, n)
        if rc:
            raise ValueError("nf4o_dequant_single rejected the shapes")
        return out

    def dequant_bnb(self, packed, a1, code2, a2, offset, numel, dtype, blocksize=64, blocksize2=256):
        packed = np.ascontiguousarray(packed, np.uint8)
        a1 = np.ascontiguousarray(a1, np.uint8)
        code2 = np.ascontiguousarray(code2, np.float32)
        a2 = np.ascontiguousarray(a2, np.float32)
        out = np.empty(numel, dtype=out_bits_dtype(dtype))
        rc = self.lib.nf4o_dequant_bnb(self._p(packed), self._p(a1), a1.size, self._p(code2),
                                       self._p(a2), a2.size, float(offset), self._p(out), dtype,
                                       numel, blocksize, blocksize2)
        if rc:
            raise ValueError("nf4o_dequant_bnb rejected the shapes")
        return out

    def dequant_bnb_single(self, packed, absmax, numel, dtype, blocksize=64):
        packed = np.ascontiguousarray(packed, np.uint8)
        absmax = np.ascontiguousarray(absmax, np.float32)
        out = np.empty(numel, dtype=out_bits_dtype(dtype))
        rc = self.lib.nf4o_dequant_bnb_single(self._p(packed), self._p(absmax), absmax.size,
                                              self._p(out), dtype, numel, blocksize)
        if rc:
            raise ValueError("nf4o_dequant_bnb_single rejected the shapes")
        return out
