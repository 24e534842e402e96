"""Property tests over shapes and quant-statistics sizes (hypothesis).

CPU (always): the three CPU restatements -- numpy, C, and the torch one with the
reference fallback's loop structure -- agree bit for bit on drawn shapes
(n % 64 != 0, odd n, padded rows), wrapping / truncated absmax counts, negative,
tiny (subnormal-product) and large nested scales, in every output dtype.  The
fixtures pin these restatements to the reference itself (test_oracle_golden.py);
this widens the input space they are compared on.

GPU (``-m gpu``): the HIP path through the drop-in API against the C oracle on the
same draws.
"""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import fallback_torch as F
import nf4_oracle as O
from _helpers import DT_CODE, assert_bits_equal, make_module, out_bits, torch_dtype


@st.composite
def cases(draw):
    m = draw(st.integers(1, 24))
    n = draw(st.one_of(st.integers(1, 300), st.sampled_from([64, 128, 192, 256, 320, 1024])))
    stride = (n + 1) // 2 + draw(st.sampled_from([0, 0, 0, 1, 7]))  # padded rows sometimes
    total_blocks = m * ((n + 63) // 64)
    nb = draw(st.one_of(st.just(None), st.integers(1, 2 * total_blocks + 3)))
    n2 = draw(st.one_of(st.just(None), st.integers(1, 40)))
    kind = draw(st.sampled_from(["uniform", "normal"]))
    scale = draw(st.sampled_from([None, 1e-30, 1e-2, 3e4]))  # subnormal products .. fp16 overflow
    dt = draw(st.sampled_from(["f16", "bf16", "f32"]))
    seed = draw(st.integers(0, 2 ** 31 - 1))
    ov = {"stride": stride, "a2_kind": kind}
    if nb is not None:
        ov["nb"] = nb
    if n2 is not None:
        ov["n2"] = n2
    if scale is not None:
        ov["a2_scale"] = scale
    return m, n, seed, ov, dt


@settings(max_examples=120, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(cases())
def test_cpu_restatements_agree(case):
    m, n, seed, ov, dt = case
    p, a1, a2, _ = O.golden_case_inputs(m, n, seed, ov)
    code = DT_CODE[dt]
    c = O.COracle().dequant_ref(p, a1, a2, m, n, code)
    assert_bits_equal(O.dequant_ref_np(p, a1, a2, m, n, code), c, dt, f"numpy {case}")
    t = F.dequant_fallback(torch.from_numpy(p), torch.from_numpy(a1), torch.from_numpy(a2), m, n, torch_dtype(dt))
    assert_bits_equal(out_bits(t), c, dt, f"fallback_torch {case}")


@pytest.mark.gpu
@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                 HealthCheck.function_scoped_fixture])
@given(cases())
def test_hip_matches_c_oracle(gpu, case):
    import nf4_triton_dequantization as N

    m, n, seed, ov, dt = case
    p, a1, a2, _ = O.golden_case_inputs(m, n, seed, ov)
    want = O.COracle().dequant_ref(p, a1, a2, m, n, DT_CODE[dt])
    out = N.triton_dequantize_nf4(make_module(p, a1, a2, m, n, dt, gpu))
    assert out.shape == (m, n) and out.dtype == torch_dtype(dt)
    assert_bits_equal(out_bits(out), want, dt, f"hip {case}")


def test_generator_is_deterministic():
    a = O.golden_case_inputs(5, 77, 123, {"nb": 9, "n2": 2, "a2_kind": "normal"})
    b = O.golden_case_inputs(5, 77, 123, {"nb": 9, "n2": 2, "a2_kind": "normal"})
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y)


# ---------------------------------------------------------------------------
# bitsandbytes semantics (parity unpinned: bitsandbytes is
# absent, so the numpy and C restatements check each other and the HIP path)
# ---------------------------------------------------------------------------
@st.composite
def bnb_cases(draw):
    bs = draw(st.sampled_from([64, 128, 256, 512, 1024, 4096]))
    bs2 = draw(st.sampled_from([256, 256, 64, 1024]))
    numel = draw(st.one_of(st.integers(1, 5000), st.sampled_from([64, 4096, 64 * 256 * 3, 64 * 1000 + 2])))
    offset = draw(st.sampled_from([0.0, 0.03125, -1.5]))
    dt = draw(st.sampled_from(["f16", "bf16", "f32"]))
    seed = draw(st.integers(0, 2 ** 31 - 1))
    return numel, bs, bs2, offset, dt, seed


def _bnb_inputs(numel, bs, bs2, seed):
    nblk = (numel + bs - 1) // bs
    packed = O.splitmix64_bytes(seed, (numel + 1) // 2, stream=1)
    a1 = O.splitmix64_bytes(seed, nblk, stream=2)
    code2 = O.normal_f32(seed, 256, stream=5)
    a2 = O.uniform_f32(seed, (nblk + bs2 - 1) // bs2, 1e-3, 1e-1, stream=3)
    return packed, a1, code2, a2


@settings(max_examples=80, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(bnb_cases())
def test_bnb_restatements_agree(case):
    numel, bs, bs2, offset, dt, seed = case
    p, a1, code2, a2 = _bnb_inputs(numel, bs, bs2, seed)
    code = DT_CODE[dt]
    c = O.COracle().dequant_bnb(p, a1, code2, a2, offset, numel, code, bs, bs2)
    assert_bits_equal(O.dequant_bnb_np(p, a1, code2, a2, offset, numel, code, bs, bs2), c, dt, f"numpy bnb {case}")


@pytest.mark.gpu
@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                 HealthCheck.function_scoped_fixture])
@given(bnb_cases())
def test_bnb_hip_matches_c_oracle(gpu, case):
    """The C ABI ``nf4_dequant_bnb`` on drawn sizes (ragged tails, every supported
    blocksize, nested block sizes, offsets) against the C restatement, bit for bit."""
    from nf4_triton_dequantization_amd import _lib

    numel, bs, bs2, offset, dt, seed = case
    p, a1, code2, a2 = _bnb_inputs(numel, bs, bs2, seed)
    want = O.COracle().dequant_bnb(p, a1, code2, a2, offset, numel, DT_CODE[dt], bs, bs2)
    t = [torch.from_numpy(v).to(gpu) for v in (p, a1, code2, a2)]
    out = torch.empty(numel, dtype=torch_dtype(dt), device=gpu)
    rc = _lib.lib().nf4_dequant_bnb(t[0].data_ptr(), t[1].data_ptr(), t[1].numel(), t[2].data_ptr(),
                                    t[3].data_ptr(), t[3].numel(), offset, out.data_ptr(), DT_CODE[dt], numel,
                                    bs, bs2, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, _lib.strerror(rc)
    assert_bits_equal(out_bits(out), want, dt, f"hip bnb {case}")
