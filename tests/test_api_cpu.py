"""Host-side logic of the drop-in API on CPU (no device work).

Mirrors what the reference's harness checks about the boundary: the import
names (benchmark.py:11), the bnb layout its ``assert_correct_bnb`` asserts
(benchmark.py:18-28), and the error behaviour of ``triton_dequantize_nf4``.
"""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import nf4_oracle as O


def test_drop_in_import_names():
    import nf4_triton_dequantization as N
    import nf4_triton_dequantization_amd as A

    assert N.triton_dequantize_nf4 is A.triton_dequantize_nf4
    assert N.reset_triton_dequantize_state is A.reset_triton_dequantize_state
    assert set(N.__all__) == {"triton_dequantize_nf4", "reset_triton_dequantize_state"}
    assert N.reset_triton_dequantize_state() is None


def _assert_correct_bnb(module, dtype):
    """The checks of reference benchmark.py:18-28, restated."""
    qs = module.weight.quant_state
    assert module.weight.dtype == torch.uint8
    assert qs.dtype == dtype
    assert qs.absmax.dtype == torch.uint8
    assert qs.code.dtype == torch.float32
    assert qs.offset.dtype == torch.float32
    assert qs.blocksize == 64
    assert qs.state2.absmax.dtype == torch.float32
    assert qs.state2.code.dtype == torch.float32
    assert qs.state2.blocksize == 256


@pytest.mark.parametrize("hd,m,dtype", [(2048, 8192, torch.float16), (1024, 4096, torch.bfloat16)])
def test_linear4bit_layout_matches_bnb(hd, m, dtype):
    from nf4_triton_dequantization_amd import Linear4bit

    torch.manual_seed(0)
    lin = Linear4bit(hd, m, bias=None, compute_dtype=dtype, compress_statistics=True, quant_type="nf4")
    _assert_correct_bnb(lin, dtype)
    assert lin.in_features == hd and lin.out_features == m
    assert lin.weight.shape == (m * hd // 2, 1)
    nb = m * hd // 64
    assert lin.weight.quant_state.absmax.shape == (nb,)
    assert lin.weight.quant_state.state2.absmax.shape == ((nb + 255) // 256,)
    assert tuple(lin.weight.quant_state.shape) == (m, hd)


def test_quantizer_packs_high_nibble_first_and_roundtrips():
    from nf4_triton_dequantization_amd.bnb_layout import NF4_CODE, quantize_nf4

    # a weight whose blocks hit every NF4 code exactly: w = code * 0.5
    idx = torch.arange(128) % 16
    w = (NF4_CODE[idx] * 0.5).reshape(2, 64)
    packed, qs = quantize_nf4(w, compress_statistics=False)
    p = packed.view(-1).numpy()
    assert p[0] == (0 << 4) | 1 and p[1] == (2 << 4) | 3  # element 0 in the high nibble
    got = O.NF4_LUT[np.stack([p >> 4, p & 15], 1).reshape(-1)] * np.repeat(qs.absmax.numpy(), 64)
    assert np.allclose(got, w.reshape(-1).numpy(), atol=0)


def test_nested_quantizer_reconstructs_weight():
    """bnb-semantics dequant of our quantizer output (numpy oracle) ~ the original weight."""
    from nf4_triton_dequantization_amd.bnb_layout import quantize_nf4

    torch.manual_seed(1)
    w = torch.randn(64, 512) * 0.02
    packed, qs = quantize_nf4(w, compress_statistics=True)
    out = O.dequant_bnb_np(packed.view(-1).numpy(), qs.absmax.numpy(), qs.state2.code.numpy(),
                           qs.state2.absmax.numpy(), float(qs.offset), w.numel(), O.F32)
    rec = out.view(np.float32).reshape(64, 512)
    rel = np.linalg.norm(rec - w.numpy()) / np.linalg.norm(w.numpy())
    assert rel < 0.12, rel


def test_dynamic_map_properties():
    from nf4_triton_dequantization_amd.bnb_layout import dynamic_map

    c = dynamic_map()
    assert c.shape == (256,) and c.dtype == torch.float32
    assert torch.all(c[1:] >= c[:-1])
    assert c.min() >= -1.0 and c.max() == 1.0 and (c == 0).any()
    assert (c > 0).sum() >= 120 and (c < 0).sum() >= 120


def _cpu_module(m=2, n=64):
    p, a1, a2 = O.make_inputs(m, n, 1)
    qs = SimpleNamespace(absmax=torch.from_numpy(a1), state2=SimpleNamespace(absmax=torch.from_numpy(a2)),
                         dtype=torch.bfloat16)
    return SimpleNamespace(weight=SimpleNamespace(data=torch.from_numpy(p).view(-1, 1), quant_state=qs),
                           out_features=m, in_features=n)


def test_cpu_tensor_raises_runtime_error():
    """The reference sends CPU tensors to Triton -> RuntimeError; so do we (no CPU path)."""
    from nf4_triton_dequantization import triton_dequantize_nf4

    with pytest.raises(RuntimeError, match="ROCm device"):
        triton_dequantize_nf4(_cpu_module())


def test_missing_state2_raises_attribute_error():
    from nf4_triton_dequantization import triton_dequantize_nf4

    mod = _cpu_module()
    mod.weight.quant_state.state2 = None
    with pytest.raises(AttributeError):
        triton_dequantize_nf4(mod)


def test_unsupported_dtype_rejected_before_device_work():
    from nf4_triton_dequantization_amd.kernel import _dtype_code

    with pytest.raises(TypeError):
        _dtype_code(torch.int8)
    assert _dtype_code(torch.float32) == 2


def test_batched_api_cpu_raises():
    from nf4_triton_dequantization_amd import dequantize_nf4_many

    with pytest.raises(RuntimeError):
        dequantize_nf4_many([_cpu_module(), _cpu_module(4, 128)])
