"""Strided (non-contiguous) packed weights and quant statistics (``-m gpu``).

The entry points make contiguous copies of strided inputs; those copies must
stay alive until the launch has been enqueued, or the caching allocator hands
their blocks to the next allocation (the output, the next weight's copy) whose
writes are queued before the kernel reads them.  Each test interleaves several
weights so a freed block WOULD be reused, then checks bit-exact / within the
GEMM tolerance against the oracle.
"""
import numpy as np
import pytest
import torch
from types import SimpleNamespace

import nf4_oracle as O
from _helpers import assert_bits_equal, out_bits

pytestmark = pytest.mark.gpu


def _strided(a: np.ndarray, dev) -> torch.Tensor:
    """Same values as `a`, as a stride-2 view of a bigger device buffer (garbage between)."""
    t = torch.from_numpy(a)
    big = torch.empty((a.size, 2), dtype=t.dtype)
    big[:, 0] = t
    big[:, 1] = t.flip(0) if t.dtype != torch.uint8 else 255 - t
    v = big.to(dev)[:, 0]
    assert not v.is_contiguous()
    return v


def _module(p, a1, a2, m, n, dt, dev):
    qs = SimpleNamespace(absmax=_strided(a1, dev), state2=SimpleNamespace(absmax=_strided(a2, dev)), dtype=dt)
    w = SimpleNamespace(data=_strided(p, dev), quant_state=qs)
    return SimpleNamespace(weight=w, out_features=m, in_features=n)


SHAPES = [(256, 1024), (128, 1024), (512, 1024)]


def test_drop_in_and_many_with_strided_inputs(coracle, gpu):
    import nf4_triton_dequantization as N
    from nf4_triton_dequantization_amd import dequantize_nf4_many

    ins = [O.make_inputs(m, n, 700 + i, a2_kind="normal") for i, (m, n) in enumerate(SHAPES)]
    mods = [_module(p, a1, a2, m, n, torch.bfloat16, gpu) for (p, a1, a2), (m, n) in zip(ins, SHAPES)]
    outs = dequantize_nf4_many(mods)
    singles = [N.triton_dequantize_nf4(mod) for mod in mods]
    torch.cuda.synchronize()
    for (p, a1, a2), (m, n), o, s in zip(ins, SHAPES, outs, singles):
        want = coracle.dequant_ref(p, a1, a2, m, n, O.BF16)
        assert_bits_equal(out_bits(o), want, "bf16", f"many {m}x{n}")
        assert_bits_equal(out_bits(s), want, "bf16", f"single {m}x{n}")


def _gemm_ref(coracle, p, a1, a2, m, n, x):
    W = coracle.dequant_ref(p, a1, a2, m, n, O.BF16)
    wf = (W.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    xf = x.float().cpu().double().numpy()
    return xf @ wf.T, np.abs(xf) @ np.abs(wf).T


@pytest.mark.parametrize("M", [1, 12, 32])
def test_linear_and_grouped_with_strided_inputs(coracle, gpu, M):
    from nf4_triton_dequantization_amd import nf4_linear, nf4_linear_grouped

    ins = [O.make_inputs(m, n, 800 + i, a2_kind="normal") for i, (m, n) in enumerate(SHAPES)]
    mods = [_module(p, a1, a2, m, n, torch.bfloat16, gpu) for (p, a1, a2), (m, n) in zip(ins, SHAPES)]
    x = torch.from_numpy(O.normal_f32(M, M * 1024, stream=9).reshape(M, 1024)).to(torch.bfloat16).to(gpu)
    grouped = nf4_linear_grouped(x, mods)
    single = [nf4_linear(x, mod) for mod in mods]
    torch.cuda.synchronize()
    for (p, a1, a2), (m, n), yg, ys in zip(ins, SHAPES, grouped, single):
        ref, mag = _gemm_ref(coracle, p, a1, a2, m, n, x)
        tol = 2.0 ** -8 * np.abs(ref) + 2.0 ** -20 * mag
        for y, what in ((yg, "grouped"), (ys, "single")):
            got = y.float().cpu().double().numpy()
            assert got.shape == ref.shape
            bad = np.abs(got - ref) > tol
            assert not bad.any(), f"{what} {m}x{n} M={M}: {bad.sum()} outside tolerance"
