"""Drop-in import name of the reference package (reference __init__.py:7-12).

``from nf4_triton_dequantization import triton_dequantize_nf4, reset_triton_dequantize_state``
resolves to the MI355X HIP implementation in ``nf4_triton_dequantization_amd``.
"""
from nf4_triton_dequantization_amd import reset_triton_dequantize_state, triton_dequantize_nf4  # noqa: F401

__all__ = ["triton_dequantize_nf4", "reset_triton_dequantize_state"]
