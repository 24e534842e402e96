"""Drop-in host side of the NF4 dequantization path (MI355X / gfx950).

Mirrors the reference's operator interface
(/root/reference/nf4_triton_dequantization/kernel_optimized.py):

* ``triton_dequantize_nf4(module)``          <- :113-139 (+ launcher :142-205)
* ``reset_triton_dequantize_state()``       <- :317-319 (no-op; no caches here either)

Same attribute reads (``module.weight.data``, ``.weight.quant_state.absmax``,
``.quant_state.state2.absmax``, ``.quant_state.dtype``, ``module.out_features``,
``module.in_features``), same value casts (qweight -> uint8 :162-163, nested
absmax -> fp32 :182), same output (new row-major ``[m, n]`` tensor of
``quant_state.dtype`` on the weight's device, :189), launched on the caller's
current stream.  A uint8 absmax takes the double-dequant kernel; any other
absmax dtype takes the single-quant kernel, exactly where the reference falls
back to ``_aggressive_pytorch_t4`` (:166-167 -> :273-274).

Error behaviour: the reference raises from torch/Triton (RuntimeError for a
tensor it cannot view or a CPU tensor -- "0 active drivers" --,
AttributeError for a missing ``state2``, ZeroDivisionError for an empty
absmax); the same exception types are raised here.  There is no CPU path and
no silent fallback: compute always goes through ``libnf4dq.so``.

Extensions beyond the reference: ``dequantize_nf4_many`` (one
launch for many weights), ``dequantize_nf4_bnb`` (bitsandbytes semantics,
parity unpinned), ``dequantize_nf4_into`` (caller-provided output) and the
consumer ``x @ W.t()`` fused: ``nf4_linear`` / ``nf4_linear_grouped``.
"""
from __future__ import annotations

import ctypes
import os
from typing import Iterable, List, Optional, Sequence

import torch

from . import _lib

_DTYPE_CODE = {torch.float16: _lib.F16, torch.bfloat16: _lib.BF16, torch.float32: _lib.F32}


BACKEND_ENV = "NF4_BACKEND"
THREADS_ENV = "NF4_CPU_THREADS"


def backend() -> str:
    """Where host (CPU) tensors go: ``NF4_BACKEND`` = ``hip`` (default) or ``cpu``.

    ``hip`` keeps the reference's behaviour: a weight on the host raises
    (the reference hands it to Triton, which has no CPU driver).  ``cpu`` runs
    host tensors through the library's own host path (``nf4_dequant_ref_cpu``,
    SURVEY §8b), bit-identical to the HIP kernels and to the reference
    fallback.  Device tensors always run on their device.  Read on every call.
    """
    b = os.environ.get(BACKEND_ENV, "hip").strip().lower() or "hip"
    if b not in ("hip", "cpu"):
        raise ValueError(f"{BACKEND_ENV}={b!r}: expected 'hip' or 'cpu'")
    return b


def cpu_threads() -> int:
    """Worker threads of the host path: ``NF4_CPU_THREADS``, else torch's intra-op thread count."""
    v = os.environ.get(THREADS_ENV, "")
    return int(v) if v.strip() else torch.get_num_threads()


def _dtype_code(dtype: torch.dtype) -> int:
    try:
        return _DTYPE_CODE[dtype]
    except KeyError:
        raise TypeError(f"unsupported quant_state.dtype {dtype}; expected float16, bfloat16, float32 "
                        f"or float64") from None


def _require_device(t: torch.Tensor) -> None:
    if t.device.type != "cuda":
        # The reference hands a CPU tensor to Triton, which raises
        # RuntimeError("0 active drivers ..."); there is no CPU path here either.
        raise RuntimeError(
            f"triton_dequantize_nf4: weight is on '{t.device}'; the NF4 HIP path needs a ROCm device tensor")


def _on_device(device: torch.device, *tensors: torch.Tensor) -> None:
    """Quant statistics must live with the packed weight (the reference hands them
    to Triton, which refuses a host tensor); never pass a host pointer to a kernel."""
    for t in tensors:
        if t.device != device:
            raise RuntimeError(f"NF4 quant state tensor on '{t.device}', packed weight on '{device}': "
                               f"all of them must be on the same ROCm device")


def _stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _as_u8_flat(q: torch.Tensor) -> torch.Tensor:
    if q.dtype != torch.uint8:
        q = q.to(torch.uint8)              # value cast, as :162-163
    return q.contiguous().view(-1)


def _prepare(module):
    """Attribute reads and casts of kernel_optimized.py:146-186."""
    weight = module.weight
    quant_state = weight.quant_state
    qweight = weight.data
    absmax = quant_state.absmax
    absmax32 = quant_state.state2.absmax    # AttributeError when state2 is None, as :151
    dtype = quant_state.dtype
    m = int(module.out_features)
    n = int(module.in_features)
    return qweight, absmax, absmax32, dtype, m, n


def _flat_ptr(t: torch.Tensor) -> tuple:
    """(tensor kept alive, data pointer, numel) of a contiguous view; copies only when needed."""
    if not t.is_contiguous():
        t = t.contiguous()
    return t, t.data_ptr(), t.numel()


def _launch(qweight, absmax, absmax32, out, m, n, code, stream) -> None:
    """Casts of kernel_optimized.py:162-186 and one C-ABI call on `stream`."""
    if qweight.dtype != torch.uint8:
        qweight = qweight.to(torch.uint8)  # value cast, as :162-163
    qweight, qp, qn = _flat_ptr(qweight)
    _on_device(qweight.device, absmax, absmax32 if absmax.dtype == torch.uint8 else absmax)
    L = _lib.lib()
    if absmax.dtype == torch.uint8:
        if absmax32.dtype != torch.float32:
            absmax32 = absmax32.to(torch.float32)  # :182
        absmax, ap, an = _flat_ptr(absmax)
        absmax32, bp, bn = _flat_ptr(absmax32)
        if an == 0 or bn == 0:
            # reference: repeats = ceil(total / 0) -> ZeroDivisionError (:175, :184)
            raise ZeroDivisionError("integer division or modulo by zero (empty absmax)")
        rc = L.nf4_dequant_ref(qp, qn, ap, an, bp, bn, out.data_ptr(), code, m, n, stream)
    else:
        # single-quant branch (:166-167 -> :273-274): absmax.view(m, -1)[:, :bpr].to(float32)
        if absmax.dtype != torch.float32:
            absmax = absmax.to(torch.float32)
        absmax, ap, an = _flat_ptr(absmax)
        rc = L.nf4_dequant_single(qp, qn, ap, an, out.data_ptr(), code, m, n, stream)
    if rc:
        _lib.check(rc, "nf4 dequantize")


def dequantize_nf4_into(qweight: torch.Tensor, absmax: torch.Tensor, absmax32: torch.Tensor,
                        out: torch.Tensor, m: int, n: int) -> torch.Tensor:
    """Dequantize into a caller-provided contiguous ``out`` ([m, n] elements, fp16/bf16/fp32)."""
    _require_device(qweight)
    code = _dtype_code(out.dtype)
    if not out.is_contiguous() or out.numel() != m * n:
        raise RuntimeError("dequantize_nf4_into: out must be a contiguous tensor of m*n elements")
    if m == 0 or n == 0:
        return out
    with torch.cuda.device(qweight.device):
        _launch(qweight, absmax, absmax32, out, m, n, code, torch.cuda.current_stream().cuda_stream)
    return out


def _launch_cpu(qweight, absmax, absmax32, out, m, n, code) -> None:
    """NF4_BACKEND=cpu: the same casts and checks, then the library's host path
    (``nf4_dequant_ref_cpu`` / ``nf4_dequant_single_cpu``, synchronous)."""
    for t in (absmax, absmax32) if absmax.dtype == torch.uint8 else (absmax,):
        if t.device.type != "cpu":
            raise RuntimeError(f"NF4 quant state tensor on '{t.device}', packed weight on the host: "
                               f"all of them must be on the same device")
    if qweight.dtype != torch.uint8:
        qweight = qweight.to(torch.uint8)  # value cast, as :162-163
    qweight, qp, qn = _flat_ptr(qweight)
    L = _lib.lib()
    threads = cpu_threads()
    if absmax.dtype == torch.uint8:
        if absmax32.dtype != torch.float32:
            absmax32 = absmax32.to(torch.float32)  # :182
        absmax, ap, an = _flat_ptr(absmax)
        absmax32, bp, bn = _flat_ptr(absmax32)
        if an == 0 or bn == 0:
            raise ZeroDivisionError("integer division or modulo by zero (empty absmax)")
        rc = L.nf4_dequant_ref_cpu(qp, qn, ap, an, bp, bn, out.data_ptr(), code, m, n, threads)
    else:
        if absmax.dtype != torch.float32:
            absmax = absmax.to(torch.float32)
        absmax, ap, an = _flat_ptr(absmax)
        rc = L.nf4_dequant_single_cpu(qp, qn, ap, an, out.data_ptr(), code, m, n, threads)
    if rc:
        _lib.check(rc, "nf4 dequantize (cpu)")


_REF = None  # bound nf4_dequant_ref (fast path: one attribute lookup less per call)
_raw_stream = torch._C._cuda_getCurrentRawStream  # device index -> hipStream_t of the current stream
_U8, _F32 = torch.uint8, torch.float32
# tensor-level fast entry (csrc/nf4_torch_ext.cpp), resolved on the first drop-in call
# (importing the package loads no native code; a missing libnf4dq.so raises there)
_EXT = None
_EXT_READY = False


def _ext():
    global _EXT, _EXT_READY
    if not _EXT_READY:
        _EXT = _lib.ext()  # raises when libnf4dq.so is missing; None when nf4ext.so is absent / unusable
        _EXT_READY = True
    return _EXT


def _dequantize(qweight, absmax, absmax32, dtype, m, n) -> torch.Tensor:
    if dtype == torch.float64:
        # the reference computes in fp32 and casts on the store (:109-110, :310):
        # fp64 output = the fp32 product, widened exactly
        return _dequantize(qweight, absmax, absmax32, torch.float32, m, n).to(torch.float64)
    code = _dtype_code(dtype)  # raise before allocating
    ext = _EXT if _EXT_READY else _ext()
    if ext is not None:
        # uint8 / uint8 / fp32 contiguous device tensors: checks, allocation, stream
        # and launch in one C++ call (None = this call needs the general path below)
        out = ext.dequant_ref(qweight, absmax, absmax32, m, n, code)
        if out is not None:
            return out
    dev = qweight.device
    if dev.type != "cuda":
        if dev.type != "cpu" or backend() != "cpu":
            _require_device(qweight)
        out = torch.empty((m, n), dtype=dtype)
        if m and n:
            _launch_cpu(qweight, absmax, absmax32, out, m, n, code)
        return out
    out = torch.empty((m, n), dtype=dtype, device=dev)
    if m == 0 or n == 0:
        return out
    idx = dev.index
    if idx == torch.cuda.current_device():
        # fast path: inputs already in the kernel's types, contiguous, on this device
        if (qweight.dtype == _U8 and absmax.dtype == _U8 and absmax32.dtype == _F32 and qweight.is_contiguous()
                and absmax.is_contiguous() and absmax32.is_contiguous() and absmax.device == dev
                and absmax32.device == dev):
            nb = absmax.numel()
            n2 = absmax32.numel()
            if nb and n2:
                global _REF
                if _REF is None:
                    _REF = _lib.lib().nf4_dequant_ref
                rc = _REF(qweight.data_ptr(), qweight.numel(), absmax.data_ptr(), nb, absmax32.data_ptr(), n2,
                          out.data_ptr(), code, m, n, _raw_stream(idx))
                if rc:
                    _lib.check(rc, "nf4 dequantize")
                return out
        _launch(qweight, absmax, absmax32, out, m, n, code, _raw_stream(idx))
    else:
        with torch.cuda.device(dev):
            _launch(qweight, absmax, absmax32, out, m, n, code, torch.cuda.current_stream().cuda_stream)
    return out


def triton_dequantize_nf4(module) -> torch.Tensor:
    """Dequantize a bitsandbytes-layout NF4 ``Linear4bit`` weight to ``[out_features, in_features]``.

    Drop-in for ``nf4_triton_dequantization.triton_dequantize_nf4``
    (kernel_optimized.py:113).  Returns a new contiguous tensor of
    ``quant_state.dtype`` on the weight's device.  Host tensors raise (as the
    reference's Triton path does) unless ``NF4_BACKEND=cpu`` selects the
    library's host path.
    """
    weight = module.weight
    quant_state = weight.quant_state
    absmax32 = quant_state.state2.absmax  # AttributeError when state2 is None, as :151
    # `.data` of an nn.Parameter builds a new tensor object per access (~0.8 us);
    # a Parameter is itself the tensor whose storage `.data` would expose
    qweight = weight if isinstance(weight, torch.Tensor) else weight.data
    m, n = int(module.out_features), int(module.in_features)
    dtype = quant_state.dtype
    ext = _EXT if _EXT_READY else _ext()
    if ext is not None:
        code = _DTYPE_CODE.get(dtype)
        if code is not None:
            # common call straight to the tensor-level entry (None = general path)
            out = ext.dequant_ref(qweight, quant_state.absmax, absmax32, m, n, code)
            if out is not None:
                return out
    return _dequantize(weight.data, quant_state.absmax, absmax32, dtype, m, n)


def reset_triton_dequantize_state() -> None:
    """No-op, as kernel_optimized.py:317-319: the path keeps no cached state."""
    return None


def dequantize_nf4_many(modules: Iterable, out: Optional[Sequence[Optional[torch.Tensor]]] = None
                        ) -> List[torch.Tensor]:
    """Dequantize several weights with as few launches as possible.

    Equivalent to ``[triton_dequantize_nf4(m) for m in modules]`` (the
    benchmark.py:68-84 pattern) but folds every uint8-absmax weight of one
    device and dtype into batched launches of up to ``NF4DQ_BATCH_MAX`` matrices.
    ``out`` (optional, one entry per module, None = allocate): caller-owned
    contiguous ``[out_features, in_features]`` tensors of ``quant_state.dtype`` on
    the weight's device, written in place and returned (a preallocated weight
    buffer reused across steps or graph replays).
    """
    modules = list(modules)
    given = list(out) if out is not None else [None] * len(modules)
    if len(given) != len(modules):
        raise ValueError("dequantize_nf4_many: one out tensor (or None) per module")
    outs: List[Optional[torch.Tensor]] = [None] * len(modules)
    groups = {}
    keep = []  # tensors referenced by descriptors must outlive the launch
    for i, mod in enumerate(modules):
        qweight, absmax, absmax32, dtype, m, n = _prepare(mod)
        o = given[i]
        if o is not None and (o.shape != (m, n) or o.dtype != dtype or o.device != qweight.device
                              or not o.is_contiguous()):
            raise RuntimeError(f"dequantize_nf4_many: out[{i}] must be a contiguous {dtype} tensor of shape "
                               f"({m}, {n}) on {qweight.device}")
        if qweight.device.type != "cuda" or absmax.dtype != torch.uint8 or dtype not in _DTYPE_CODE:
            # host tensors (NF4_BACKEND=cpu, or the reference's error), single-quant
            # absmax, fp64 output: one call each
            r = triton_dequantize_nf4(mod)
            outs[i] = o.copy_(r) if o is not None else r
            continue
        code = _dtype_code(dtype)
        out_t = o if o is not None else torch.empty((m, n), dtype=dtype, device=qweight.device)
        outs[i] = out_t
        if m == 0 or n == 0:
            continue
        q = _as_u8_flat(qweight)
        _on_device(q.device, absmax, absmax32)
        a1 = absmax.contiguous().view(-1)
        a2 = absmax32.reshape(-1)
        a2 = (a2 if a2.dtype == torch.float32 else a2.to(torch.float32)).contiguous()
        if a1.numel() == 0 or a2.numel() == 0:
            raise ZeroDivisionError("integer division or modulo by zero (empty absmax)")
        keep.extend((q, a1, a2))
        d = _lib.MatrixDesc(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                            out_t.data_ptr(), m, n)
        groups.setdefault((q.device, code), []).append(d)
    L = _lib.lib()
    for (device, code), descs in groups.items():
        arr = (_lib.MatrixDesc * len(descs))(*descs)
        with torch.cuda.device(device):
            rc = L.nf4_dequant_ref_batched(arr, len(descs), code, _stream_ptr(device))
        _lib.check(rc, "nf4 batched dequantize")
    # Temporaries in `keep` (value casts) were allocated on the stream the
    # launches use, so the caching allocator's stream-ordered reuse already
    # protects them; no record_stream needed (and it would break graph capture).
    del keep
    return outs  # type: ignore[return-value]


def dequantize_nf4_bnb(module) -> torch.Tensor:
    """bitsandbytes ``dequantize_4bit`` semantics (parity unpinned).

    Reads ``quant_state.{absmax, code?, offset, blocksize, shape, dtype}`` and, when
    nested, ``state2.{absmax, code, blocksize}``; output has ``quant_state.shape``.
    """
    weight = module.weight
    qs = weight.quant_state
    _require_device(weight.data)
    q = _as_u8_flat(weight.data)
    shape = tuple(qs.shape) if getattr(qs, "shape", None) is not None else (int(module.out_features),
                                                                            int(module.in_features))
    numel = 1
    for s in shape:
        numel *= int(s)
    code = _dtype_code(qs.dtype)
    out = torch.empty(shape, dtype=qs.dtype, device=q.device)
    if numel == 0:
        return out
    bs = int(qs.blocksize)
    with torch.cuda.device(q.device):  # the launch's device = the weight's (not the current one)
        rc = _launch_bnb(q, qs, out, code, numel, bs)
    _lib.check(rc, "nf4 bnb dequantize")
    return out


def _launch_bnb(q, qs, out, code, numel, bs) -> int:
    L = _lib.lib()
    stream = _stream_ptr(q.device)
    nested = getattr(qs, "state2", None) is not None and qs.absmax.dtype == torch.uint8
    if nested:
        _on_device(q.device, qs.absmax, qs.state2.code, qs.state2.absmax)
        a1 = qs.absmax.contiguous().view(-1)
        code2 = qs.state2.code.to(torch.float32).contiguous()
        a2 = qs.state2.absmax.to(torch.float32).contiguous().view(-1)
        off = qs.offset
        off = float(off.item()) if torch.is_tensor(off) else float(off or 0.0)
        rc = L.nf4_dequant_bnb(q.data_ptr(), a1.data_ptr(), a1.numel(), code2.data_ptr(), a2.data_ptr(),
                               a2.numel(), ctypes.c_float(off), out.data_ptr(), code, numel, bs,
                               int(qs.state2.blocksize), stream)
    else:
        _on_device(q.device, qs.absmax)
        am = qs.absmax.to(torch.float32).contiguous().view(-1)
        rc = L.nf4_dequant_bnb_single(q.data_ptr(), am.data_ptr(), am.numel(), out.data_ptr(), code, numel,
                                      bs, stream)
    return rc


# (device index, raw stream handle) -> (workspace, the torch stream object): holding the
# stream object keeps a torch-created stream alive for the cache's lifetime, so the
# check below never hands HIP a dangling handle (an ExternalStream's owner must keep
# its stream alive while nf4_linear has a workspace for it, or call
# release_gemm_workspaces() first)
_GEMM_WS = {}


def _same_device(x: torch.Tensor, w: torch.Tensor) -> None:
    # what `x @ W.t()` raises for tensors on different devices (never hand a host
    # or foreign-device pointer to the kernel)
    if x.device != w.device:
        raise RuntimeError(f"Expected all tensors to be on the same device, but found at least two devices, "
                           f"{w.device} and {x.device}!")


def _gemm_workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    """Zero-filled split-K workspace, one per (device, stream), grown on demand.

    The fused kernel leaves its ticket counters at 0 after every call, so the
    buffer stays valid; a new stream gets its own (calls on different streams
    may run concurrently and must not share counters).
    """
    stream = torch.cuda.current_stream(device)
    key = (device.index, stream.cuda_stream)
    ent = _GEMM_WS.get(key)
    ws = ent[0] if ent is not None else None
    if ws is None or ws.numel() < nbytes:
        ws = torch.zeros(max(nbytes, 1 << 16), dtype=torch.uint8, device=device)
        _GEMM_WS[key] = (ws, stream)
    return ws


def release_gemm_workspaces() -> None:
    """Forget every cached split-K workspace: for callers that destroy their own external
    streams.  Each workspace's sticky error word is read first (which also waits for its
    stream), so a split-K timeout since the last ``check_gemm_workspaces()`` is not lost
    with the workspace: the cache is cleared either way, then RuntimeError is raised as
    ``check_gemm_workspaces`` would."""
    try:
        check_gemm_workspaces()
    finally:
        _GEMM_WS.clear()


def check_gemm_workspaces() -> None:
    """Raise if a fused-GEMM split-K reduction gave up waiting since the last check.

    Waits for every stream that owns one of ``nf4_linear``'s cached workspaces and reads
    its sticky error word (``nf4_gemm_check_workspace``); a stalled K slice
    makes the reducer emit NaN for the missing partial and set the word.  The library
    re-zeroes such a workspace, so the next call starts clean.  Raises RuntimeError
    naming the device and stream; returns None when every workspace is clean.
    """
    bad = []
    L = _lib.lib() if _GEMM_WS else None
    for (dev_index, handle), (ws, stream) in list(_GEMM_WS.items()):
        with torch.cuda.device(dev_index):  # the HIP calls run on the workspace's device
            rc = L.nf4_gemm_check_workspace(ws.data_ptr(), ws.numel(), stream.cuda_stream)
        if rc:
            bad.append(f"cuda:{dev_index} stream {handle:#x}: {_lib.strerror(rc)}")
    if bad:
        raise RuntimeError("nf4 fused GEMM: " + "; ".join(bad))


def nf4_linear(x: torch.Tensor, module, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x @ W.t() (+ bias)`` for an NF4 ``Linear4bit`` weight W (reference semantics).

    The consumer of the reference harness (benchmark.py:61-66,
    ``X @ triton_dequantize_nf4(W).t()``).  Decode-shaped inputs (at most
    ``NF4DQ_GEMM_MAX_M`` rows, N % 64 == 0, K % 128 == 0, uint8 absmax) run the
    fused kernel: the 4-bit weight is read once and dequantized in registers
    into exactly the bf16/fp16 values ``triton_dequantize_nf4`` returns, then
    multiplied on MFMA with fp32 accumulation.  Anything else dequantizes with
    the HIP kernel and multiplies with torch (hipBLASLt).  Output dtype =
    ``quant_state.dtype``; ``x`` is cast to it first, as the reference harness's
    inputs already are.
    """
    qweight, absmax, absmax32, dtype, m, n = _prepare(module)
    if qweight.device.type != "cuda" and backend() != "cpu":
        _require_device(qweight)
    _same_device(x, qweight)
    N, K = m, n
    if x.shape[-1] != K:
        raise RuntimeError(f"nf4_linear: x has {x.shape[-1]} features, weight expects {K}")
    lead = x.shape[:-1]
    M = x.numel() // K if K else 0
    fused = (qweight.device.type == "cuda" and dtype in (torch.float16, torch.bfloat16)
             and absmax.dtype == torch.uint8 and 0 < M <= _lib.GEMM_MAX_M
             and N % 64 == 0 and K % 128 == 0 and qweight.numel() * qweight.element_size() == N * K // 2
             and qweight.dtype == torch.uint8)
    if not fused:
        w = triton_dequantize_nf4(module)
        y = x.to(dtype) @ w.t()
    else:
        xc = x.reshape(M, K)
        if xc.dtype != dtype:
            xc = xc.to(dtype)
        xc = xc.contiguous()
        y = torch.empty((M, N), dtype=dtype, device=qweight.device)
        _on_device(qweight.device, absmax, absmax32)
        L = _lib.lib()
        ws_bytes = L.nf4_gemm_workspace_bytes(M, N, K)
        with torch.cuda.device(qweight.device):
            ws = _gemm_workspace(qweight.device, ws_bytes) if ws_bytes else None
            q, qp, qn = _flat_ptr(qweight)
            a1, ap, an = _flat_ptr(absmax)
            a2 = absmax32 if absmax32.dtype == torch.float32 else absmax32.to(torch.float32)
            a2, bp, bn = _flat_ptr(a2)
            if an == 0 or bn == 0:
                raise ZeroDivisionError("integer division or modulo by zero (empty absmax)")
            rc = L.nf4_gemm_ref(xc.data_ptr(), M, qp, qn, ap, an, bp, bn, y.data_ptr(), _dtype_code(dtype), N, K,
                                ws.data_ptr() if ws is not None else None, ws_bytes,
                                torch.cuda.current_stream().cuda_stream)
        _lib.check(rc, "nf4 fused gemm")
        y = y.reshape(*lead, N)
    if bias is not None:
        y = y + bias.to(y.dtype)
    return y.reshape(*lead, N)


def nf4_linear_grouped(x: torch.Tensor, modules: Sequence, biases: Optional[Sequence] = None) -> List[torch.Tensor]:
    """``[x @ W_i.t() (+ b_i)]`` for NF4 weights W_i that share the input x (q/k/v, gate/up).

    One fused launch for all of them (``nf4_gemm_ref_grouped``) when every
    weight meets ``nf4_linear``'s fused-path rules, has the same ``in_features``
    and output dtype, and there are at most ``GEMM_GROUP_MAX`` of them;
    otherwise each goes through ``nf4_linear``.  Results are the same values
    ``nf4_linear`` gives per weight (same dequantized weights, fp32
    accumulation; the summation order may differ).
    """
    modules = list(modules)
    biases = list(biases) if biases is not None else [None] * len(modules)
    if len(biases) != len(modules):
        raise ValueError("nf4_linear_grouped: one bias (or None) per module")
    if not modules:
        return []
    preps = [_prepare(mod) for mod in modules]
    K = x.shape[-1]
    lead = x.shape[:-1]
    M = x.numel() // K if K else 0
    dtype = preps[0][3]
    dev = preps[0][0].device
    grouped = 1 < len(modules) <= _lib.GEMM_GROUP_MAX and 0 < M <= _lib.GEMM_MAX_M and K % 128 == 0
    for (q, a1, _a2, dt, m, n) in preps:
        grouped = grouped and (dt == dtype and dt in (torch.float16, torch.bfloat16) and n == K and m % 64 == 0
                               and a1.dtype == torch.uint8 and q.dtype == torch.uint8 and q.device == dev
                               and q.numel() == m * K // 2)
    if not grouped:
        return [nf4_linear(x, mod, bias=b) for mod, b in zip(modules, biases)]
    _require_device(preps[0][0])
    _same_device(x, preps[0][0])
    xc = x.reshape(M, K)
    if xc.dtype != dtype:
        xc = xc.to(dtype)
    xc = xc.contiguous()
    ys, keep = [], []
    mats = (_lib.GemmMat * len(modules))()
    for i, (q, a1, a2, _dt, m, _n) in enumerate(preps):
        _on_device(dev, a1, a2)
        y = torch.empty((M, m), dtype=dtype, device=dev)
        # the contiguous copies (when q / a1 / a2 are strided views) must outlive the
        # launch: the caching allocator would hand their blocks to the next torch.empty
        qc, qp, qn = _flat_ptr(q)
        a1c, ap, an = _flat_ptr(a1)
        a2f = a2 if a2.dtype == torch.float32 else a2.to(torch.float32)
        a2f, bp, bn = _flat_ptr(a2f)
        if an == 0 or bn == 0:
            raise ZeroDivisionError("integer division or modulo by zero (empty absmax)")
        keep.extend((qc, a1c, a2f))
        mats[i] = _lib.GemmMat(qp, qn, ap, an, bp, bn, y.data_ptr(), m)
        ys.append(y)
    L = _lib.lib()
    with torch.cuda.device(dev):
        ws_bytes = L.nf4_gemm_grouped_workspace_bytes(M, K, mats, len(modules), None)
        ws = _gemm_workspace(dev, ws_bytes) if ws_bytes else None
        rc = L.nf4_gemm_ref_grouped(xc.data_ptr(), M, K, mats, len(modules), _dtype_code(dtype),
                                    ws.data_ptr() if ws is not None else None, ws_bytes, None,
                                    torch.cuda.current_stream().cuda_stream)
    _lib.check(rc, "nf4 fused grouped gemm")
    out = []
    for y, b, (_q, _a1, _a2, _dt, m, _n) in zip(ys, biases, preps):
        if b is not None:
            y = y + b.to(y.dtype)
        out.append(y.reshape(*lead, m))
    return out
