"""MI355X-native NF4 double-dequantization (gfx950 HIP kernels behind a C ABI).

Public API mirrors the reference package ``nf4_triton_dequantization``
(/root/reference/nf4_triton_dequantization/__init__.py:7-12):

    from nf4_triton_dequantization_amd import triton_dequantize_nf4, reset_triton_dequantize_state

The alias package ``nf4_triton_dequantization`` (repo root) re-exports the same
names so existing callers (benchmark.py:11) import it unchanged.
"""
from .kernel import (  # noqa: F401
    check_gemm_workspaces,
    dequantize_nf4_bnb,
    dequantize_nf4_into,
    dequantize_nf4_many,
    nf4_linear,
    nf4_linear_grouped,
    release_gemm_workspaces,
    reset_triton_dequantize_state,
    triton_dequantize_nf4,
)
from .bnb_layout import Linear4bit, Params4bit, QuantState, quantize_nf4  # noqa: F401
from .checkpoint import load_nf4_safetensors, save_nf4_safetensors  # noqa: F401

__all__ = ["triton_dequantize_nf4", "reset_triton_dequantize_state", "dequantize_nf4_many",
           "dequantize_nf4_bnb", "dequantize_nf4_into", "nf4_linear", "nf4_linear_grouped", "check_gemm_workspaces",
           "release_gemm_workspaces", "Linear4bit",
           "Params4bit", "QuantState", "quantize_nf4", "load_nf4_safetensors", "save_nf4_safetensors"]
__version__ = "0.1.0"
