"""ctypes binding of the C ABI in include/nf4_dequant.h (libnf4dq.so, gfx950).

The library is loaded after ``import torch`` so that it binds to the HIP runtime
torch already mapped (same SONAME ``libamdhip64.so.7``): one HIP runtime per
process.  There is no fallback: if the library is missing or fails to load,
``lib()`` raises, and so does every product entry point that needs it.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  -- must precede the CDLL load (shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
# NF4DQ_LIB_PATH: load a diagnostic build of the same library instead (tools/Makefile);
# unset in every product / test / bench run (when set, the tensor-level entry is not
# loaded, so every call goes to that build)
LIB_PATH = os.environ.get("NF4DQ_LIB_PATH") or os.path.join(_HERE, "_lib", "libnf4dq.so")
EXT_PATH = os.path.join(_HERE, "_lib", "nf4ext.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "nf4_dequant.h")

F16 = 0
BF16 = 1
F32 = 2

OK = 0
ERR_ARG = 1
ERR_SHAPE = 2
ERR_TOO_LARGE = 3
ERR_SPLITK_TIMEOUT = 4
ERR_HIP_BASE = 1000

BATCH_MAX = 24
GEMM_MAX_M = 32


class MatrixDesc(ctypes.Structure):
    """nf4_matrix_desc (include/nf4_dequant.h)."""

    _fields_ = [
        ("packed", ctypes.c_void_p),
        ("packed_len", ctypes.c_int64),
        ("absmax_q", ctypes.c_void_p),
        ("nb", ctypes.c_int64),
        ("absmax2", ctypes.c_void_p),
        ("n2", ctypes.c_int64),
        ("out", ctypes.c_void_p),
        ("m", ctypes.c_int64),
        ("n", ctypes.c_int64),
    ]


class LaunchCfg(ctypes.Structure):
    """nf4_launch_cfg (include/nf4_dequant.h)."""

    _fields_ = [
        ("tile_dwords", ctypes.c_int32),
        ("blocks_per_cu", ctypes.c_int32),
        ("nontemporal", ctypes.c_int32),
        ("flags", ctypes.c_int32),
    ]


CFG_ROWS = 1    # NF4DQ_CFG_ROWS: the one-thread-per-byte general kernel
CFG_CHUNKS = 2  # NF4DQ_CFG_CHUNKS: the chunk / piece kernels' path, even for a flat-eligible matrix


GEMM_K128 = 1
GEMM_STREAM = 2
GEMM_PERSIST = 3
GEMM_XS = 4
GEMM_XR = 5
GEMM_SK = 6  # retired in round 6: rejected with ERR_ARG
GEMM_GEMV = 7  # the decode GEMV (M = 1, K % 2048 == 0)


GEMM_GROUP_MAX = 8


class GemmMat(ctypes.Structure):
    """nf4_gemm_mat (include/nf4_dequant.h)."""

    _fields_ = [("packed", ctypes.c_void_p), ("packed_len", ctypes.c_int64), ("absmax_q", ctypes.c_void_p),
                ("nb", ctypes.c_int64), ("absmax2", ctypes.c_void_p), ("n2", ctypes.c_int64),
                ("y", ctypes.c_void_p), ("N", ctypes.c_int64)]


class GemmCfg(ctypes.Structure):
    """nf4_gemm_cfg (include/nf4_dequant.h)."""

    _fields_ = [("kernel", ctypes.c_int32), ("waves", ctypes.c_int32), ("depth", ctypes.c_int32),
                ("ksplit", ctypes.c_int32), ("strips", ctypes.c_int32)]


# name -> (restype, argtypes); every symbol include/nf4_dequant.h declares.
_P, _I64, _I32, _F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
SIGNATURES = {
    "nf4_dequant_ref": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _I64, _P, _I32, _I64, _I64, _P]),
    "nf4_dequant_single": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _I32, _I64, _I64, _P]),
    "nf4_dequant_ref_cpu": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _I64, _P, _I32, _I64, _I64, _I32]),
    "nf4_dequant_single_cpu": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _I32, _I64, _I64, _I32]),
    "nf4_dequant_ref_batched": (ctypes.c_int, [ctypes.POINTER(MatrixDesc), _I32, _I32, _P]),
    "nf4_dequant_bnb": (ctypes.c_int, [_P, _P, _I64, _P, _P, _I64, _F, _P, _I32, _I64, _I32, _I32, _P]),
    "nf4_dequant_bnb_single": (ctypes.c_int, [_P, _P, _I64, _P, _I32, _I64, _I32, _P]),
    "nf4_dequant_ref_cfg": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _I64, _P, _I32, _I64, _I64,
                                           ctypes.POINTER(LaunchCfg), _P]),
    "nf4_gemm_workspace_bytes": (ctypes.c_size_t, [_I64, _I64, _I64]),
    "nf4_gemm_ref": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I32, _I64, _I64, _P, ctypes.c_size_t,
                                    _P]),
    "nf4_gemm_workspace_bytes_cfg": (ctypes.c_size_t, [_I64, _I64, _I64, ctypes.POINTER(GemmCfg)]),
    "nf4_gemm_ref_cfg": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I32, _I64, _I64, _P,
                                        ctypes.c_size_t, ctypes.POINTER(GemmCfg), _P]),
    "nf4_gemm_grouped_workspace_bytes": (ctypes.c_size_t, [_I64, _I64, ctypes.POINTER(GemmMat), _I32,
                                                           ctypes.POINTER(GemmCfg)]),
    "nf4_gemm_ref_grouped": (ctypes.c_int, [_P, _I64, _I64, ctypes.POINTER(GemmMat), _I32, _I32, _P, ctypes.c_size_t,
                                            ctypes.POINTER(GemmCfg), _P]),
    "nf4_gemm_check_workspace": (ctypes.c_int, [_P, ctypes.c_size_t, _P]),
    "nf4_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "nf4_version": (ctypes.c_char_p, []),
}

_lock = threading.Lock()
_lib = None


def lib() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"nf4 HIP library not built: {LIB_PATH} is missing "
                    "(run `python __graft_entry__.py build` or `make -C nf4_triton_dequantization_amd`)")
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


_ext = None
_ext_tried = False


def ext():
    """The tensor-level fast entry (``_lib/nf4ext.so``, csrc/nf4_torch_ext.cpp), or None:
    callers then take the ctypes route to the same kernels.

    None when the extension is not built, when it fails to load (a stale build or a
    torch ABI mismatch: a warning names the error), and when ``NF4DQ_LIB_PATH``
    selects another build of the C ABI -- the extension links the product
    ``_lib/libnf4dq.so`` through its rpath, so loading it then would put two copies
    of the library in the process and the drop-in would run the other one.
    Raises like ``lib()`` when the C ABI itself is missing.
    """
    global _ext, _ext_tried
    if not _ext_tried:
        lib()  # the C ABI first (the extension links it; one copy per process); takes _lock itself
        with _lock:
            if not _ext_tried:
                if os.path.exists(EXT_PATH) and not os.environ.get("NF4DQ_LIB_PATH"):
                    import importlib.util

                    try:
                        spec = importlib.util.spec_from_file_location("nf4ext", EXT_PATH)
                        mod = importlib.util.module_from_spec(spec)
                        spec.loader.exec_module(mod)
                        _ext = mod
                    except (ImportError, OSError) as e:
                        import warnings

                        warnings.warn(f"nf4ext.so did not load ({e}); the drop-in uses the ctypes route "
                                      f"to the same kernels", RuntimeWarning, stacklevel=2)
                        _ext = None
                _ext_tried = True
    return _ext


def strerror(code: int) -> str:
    return lib().nf4_strerror(int(code)).decode()


def check(code: int, what: str) -> None:
    if code != OK:
        raise RuntimeError(f"{what} failed: {strerror(code)} (code {code})")
