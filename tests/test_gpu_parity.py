"""HIP path vs the oracle on an MI355X (``-m gpu``), through the product API and C ABI.

Bar: bit-exact for fp16 / bf16 / fp32 outputs (NaN payloads excepted, see
_helpers.assert_bits_equal); the BASELINE tolerance (1e-3 fp16 max-abs) is
reported on top and is implied by bit-exactness.  Full-size configs are pinned
to the sha256 of the REFERENCE's own output (tests/golden/manifest.json).
"""
import ctypes

import numpy as np
import pytest
import torch

import nf4_oracle as O
from _helpers import (DT_CODE, assert_bits_equal, big_samples, load_case, make_module, max_abs_diff, out_bits,
                      sha, torch_dtype)

pytestmark = pytest.mark.gpu

TOL_F16_MAX_ABS = 1e-3  # BASELINE.json north_star tolerance


def _api():
    import nf4_triton_dequantization as N  # the drop-in import name

    return N


def test_golden_small_cases_bit_exact(manifest, gpu):
    N = _api()
    for name, e in manifest["cases"].items():
        if "file" not in e:
            continue
        z = load_case(e)
        m, n, dt = e["m"], e["n"], e["dtype"]
        absmax = z["absmax_f32"] if "absmax_f32" in z else z["a1"]
        mod = make_module(z["packed"], absmax, z["a2"], m, n, dt, gpu, a2_f16=z.get("a2_f16"))
        out = N.triton_dequantize_nf4(mod)
        assert out.shape == (m, n) and out.dtype == torch_dtype(dt) and out.is_contiguous()
        assert out.device == gpu
        got = out_bits(out)
        assert_bits_equal(got, z["out_bits"], dt, name)
        if dt == "f16":
            assert max_abs_diff(got, z["out_bits"], dt) <= TOL_F16_MAX_ABS


# every full-size case of the manifest: C1, C2, C4's fp16 leg, C5's per-GPU 8192^2
# unit and each distinct C3 shape (Llama-3-8B and Llama-2-7B linears)
@pytest.mark.parametrize("name", ["C1_1024x1024_f16", "C2_4096x4096_bf16", "c64x11008_bf16",
                                  "c1024x4096_f16_neg", "C4_4096x4096_f16", "C5_8192x8192_bf16",
                                  "C3_1024x4096_bf16", "C3_14336x4096_bf16", "C3_4096x14336_bf16",
                                  "C3b_11008x4096_bf16", "C3b_4096x11008_bf16"])
def test_full_size_matches_reference_digest(manifest, gpu, name):
    e = manifest["cases"][name]
    m, n, dt = e["m"], e["n"], e["dtype"]
    p, a1, a2, _ = O.golden_case_inputs(m, n, e["seed"], e["overrides"])
    out = _api().triton_dequantize_nf4(make_module(p, a1, a2, m, n, dt, gpu))
    got = out_bits(out)
    idx, bits = big_samples(name)
    assert np.array_equal(got.reshape(-1)[idx], bits), name
    assert sha(got) == e["sha256"], name


SHAPES = [(1, 64), (3, 128), (17, 192), (64, 256), (5, 77), (9, 1000), (2, 11008), (33, 4096), (128, 320),
          (7, 64 * 33), (256, 256), (1, 2)]


@pytest.mark.parametrize("dt", ["f16", "bf16", "f32"])
@pytest.mark.parametrize("m,n", SHAPES)
def test_random_shapes_vs_c_oracle(coracle, gpu, m, n, dt):
    seed = m * 1000 + n
    for ov in ({}, {"nb": 7, "n2": 3}, {"a2_kind": "normal"}):
        p, a1, a2, _ = O.golden_case_inputs(m, n, seed, dict(ov, stride=(n + 1) // 2))
        want = coracle.dequant_ref(p, a1, a2, m, n, DT_CODE[dt])
        out = _api().triton_dequantize_nf4(make_module(p, a1, a2, m, n, dt, gpu))
        assert_bits_equal(out_bits(out), want, dt, f"{m}x{n} {dt} {ov}")


def test_padded_rows_and_unaligned_views(coracle, gpu):
    """Row stride > n/2 and a packed view at an odd byte offset take the chunk kernel."""
    m, n = 6, 256
    p, a1, a2, _ = O.golden_case_inputs(m, n, 5, {"stride": 130})
    want = coracle.dequant_ref(p, a1, a2, m, n, O.BF16)
    got = _api().triton_dequantize_nf4(make_module(p, a1, a2, m, n, "bf16", gpu))
    assert_bits_equal(out_bits(got), want, "bf16", "padded")
    # odd offset: slice of a bigger buffer
    p2, a1, a2, _ = O.golden_case_inputs(m, n, 6, {})
    big = torch.zeros(p2.size + 1, dtype=torch.uint8, device=gpu)
    big[1:] = torch.from_numpy(p2).to(gpu)
    mod = make_module(p2, a1, a2, m, n, "f16", gpu)
    mod.weight.data = big[1:].view(-1, 1)
    want = coracle.dequant_ref(p2, a1, a2, m, n, O.F16)
    assert_bits_equal(out_bits(_api().triton_dequantize_nf4(mod)), want, "f16", "odd offset")


def test_single_quant_branch(coracle, gpu):
    for (m, n, extra) in ((12, 256, 0), (6, 200, 3), (64, 4096, 1)):
        p, a1, a2, single = O.golden_case_inputs(m, n, m + n, {"single": extra})
        for dt in ("f16", "bf16", "f32"):
            want = coracle.dequant_single(p, single, m, n, DT_CODE[dt])
            mod = make_module(p, single, a2, m, n, dt, gpu)
            assert_bits_equal(out_bits(_api().triton_dequantize_nf4(mod)), want, dt, f"single {m}x{n}")
    # bf16 absmax is value-cast to fp32 first (:274)
    m, n = 8, 128
    p, a1, a2, single = O.golden_case_inputs(m, n, 3, {"single": 0})
    s16 = torch.from_numpy(single).to(torch.bfloat16)
    want = coracle.dequant_single(p, s16.float().numpy(), m, n, O.F16)
    mod = make_module(p, single, a2, m, n, "f16", gpu)
    mod.weight.quant_state.absmax = s16.to(gpu)
    assert_bits_equal(out_bits(_api().triton_dequantize_nf4(mod)), want, "f16", "bf16 absmax")


def test_non_uint8_qweight_is_value_cast(coracle, gpu):
    m, n = 4, 128
    p, a1, a2, _ = O.golden_case_inputs(m, n, 9, {})
    mod = make_module(p, a1, a2, m, n, "bf16", gpu)
    mod.weight.data = torch.from_numpy(p.astype(np.int16)).to(gpu).view(-1, 1)  # .to(uint8) :162-163
    want = coracle.dequant_ref(p, a1, a2, m, n, O.BF16)
    assert_bits_equal(out_bits(_api().triton_dequantize_nf4(mod)), want, "bf16", "int16 qweight")


def test_empty_and_error_behaviour(gpu):
    N = _api()
    p, a1, a2, _ = O.golden_case_inputs(2, 64, 1, {})
    mod = make_module(p, a1, a2, 0, 64, "bf16", gpu)
    assert N.triton_dequantize_nf4(mod).shape == (0, 64)
    bad = make_module(p, a1, a2, 3, 64, "bf16", gpu)  # 64 packed bytes cannot be viewed as (3, -1)
    with pytest.raises(RuntimeError):
        N.triton_dequantize_nf4(bad)
    mod = make_module(p, a1[:0], a2, 2, 64, "bf16", gpu)
    with pytest.raises(ZeroDivisionError):
        N.triton_dequantize_nf4(mod)
    mod = make_module(p, a1, a2, 2, 64, "bf16", gpu)
    mod.weight.quant_state.state2 = None
    with pytest.raises(AttributeError):
        N.triton_dequantize_nf4(mod)


def test_three_stream_pattern(coracle, gpu):
    """benchmark.py:68-84: three weights dequantized on three fresh streams."""
    N = _api()
    shapes = [(1024, 4096), (4096, 1024), (512, 2048)]
    mods, wants = [], []
    for i, (m, n) in enumerate(shapes):
        p, a1, a2, _ = O.golden_case_inputs(m, n, 100 + i, {})
        mods.append(make_module(p, a1, a2, m, n, "bf16", gpu))
        wants.append(coracle.dequant_ref(p, a1, a2, m, n, O.BF16))
    for _ in range(3):
        streams = [torch.cuda.Stream() for _ in mods]
        outs = []
        for s, mod in zip(streams, mods):
            with torch.cuda.stream(s):
                outs.append(N.triton_dequantize_nf4(mod).t())
        torch.cuda.synchronize()
        for o, w in zip(outs, wants):
            assert_bits_equal(out_bits(o.t()), w, "bf16", "3-stream")


def test_batched_matches_single_calls(coracle, gpu):
    from nf4_triton_dequantization_amd import dequantize_nf4_many

    shapes = [(64, 4096), (1024, 64), (5, 77), (33, 11008), (8, 96)] * 6  # 30 > NF4DQ_BATCH_MAX
    mods, wants = [], []
    for i, (m, n) in enumerate(shapes):
        p, a1, a2, _ = O.golden_case_inputs(m, n, 200 + i, {"stride": (n + 1) // 2})
        mods.append(make_module(p, a1, a2, m, n, "f16", gpu))
        wants.append(coracle.dequant_ref(p, a1, a2, m, n, O.F16))
    outs = dequantize_nf4_many(mods)
    torch.cuda.synchronize()
    for i, (o, w) in enumerate(zip(outs, wants)):
        assert_bits_equal(out_bits(o), w, "f16", f"batched #{i}")
    # the same into caller-owned outputs (every other one preallocated, stale contents)
    bufs = [torch.full((m, n), float("nan"), dtype=torch.float16, device=gpu) if i % 2 == 0 else None
            for i, (m, n) in enumerate(shapes)]
    outs = dequantize_nf4_many(mods, out=bufs)
    torch.cuda.synchronize()
    for i, (o, w) in enumerate(zip(outs, wants)):
        assert bufs[i] is None or o is bufs[i]
        assert_bits_equal(out_bits(o), w, "f16", f"batched into #{i}")


# the one launch knob the library keeps (include/nf4_dequant.h): the grid cap
# (persistent waves walking several tiles; 1 and 3 workgroups per CU give odd and
# even tile counts, so both loop exits run); flags 0 (the kernel-choice flags: test_gpu_chunks.py)
@pytest.mark.parametrize("cfg", [(4, 0, 1, 0), (4, 1, 1, 0), (4, 2, 1, 0), (4, 3, 1, 0), (4, 8, 1, 0)])
def test_launch_configs_identical(coracle, gpu, cfg):
    from nf4_triton_dequantization_amd import _lib

    m, n = 1024, 4096 + 64 * 3  # partial last tile
    p, a1, a2, _ = O.golden_case_inputs(m, n, 77, {})
    want = coracle.dequant_ref(p, a1, a2, m, n, O.BF16)
    q = torch.from_numpy(p).to(gpu)
    t1 = torch.from_numpy(a1).to(gpu)
    t2 = torch.from_numpy(a2).to(gpu)
    out = torch.empty((m, n), dtype=torch.bfloat16, device=gpu)
    c = _lib.LaunchCfg(*cfg)
    rc = _lib.lib().nf4_dequant_ref_cfg(q.data_ptr(), q.numel(), t1.data_ptr(), t1.numel(), t2.data_ptr(),
                                        t2.numel(), out.data_ptr(), _lib.BF16, m, n, ctypes.byref(c),
                                        torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    assert_bits_equal(out_bits(out), want, "bf16", f"cfg {cfg}")


def test_bnb_semantics_vs_oracle_and_roundtrip(coracle, gpu):
    """bitsandbytes mode (parity unpinned): matches the numpy/C restatement bit for bit
    and reconstructs the quantized weight to NF4 accuracy."""
    from nf4_triton_dequantization_amd import Linear4bit, dequantize_nf4_bnb

    torch.manual_seed(0)
    for (o, i, nested) in ((256, 512, True), (96, 320, True), (128, 256, False), (3, 70, True)):
        w = torch.randn(o, i, device=gpu) * 0.02
        lin = Linear4bit(i, o, compute_dtype=torch.bfloat16, compress_statistics=nested, weight=w)
        qs = lin.weight.quant_state
        out = dequantize_nf4_bnb(lin)
        assert out.shape == (o, i) and out.dtype == torch.bfloat16
        p = lin.weight.data.view(-1).cpu().numpy()
        if nested:
            want = coracle.dequant_bnb(p, qs.absmax.cpu().numpy(), qs.state2.code.cpu().numpy(),
                                       qs.state2.absmax.cpu().numpy(), float(qs.offset.item()), o * i, O.BF16)
        else:
            want = coracle.dequant_bnb_single(p, qs.absmax.cpu().numpy(), o * i, O.BF16)
        assert_bits_equal(out_bits(out).reshape(-1), want, "bf16", f"bnb {o}x{i}")
        rel = ((out.float() - w).norm() / w.norm()).item()
        assert rel < 0.12, rel  # 4-bit NF4 of a gaussian: ~0.09-0.1 rel-L2


def test_linear4bit_layout_and_forward(gpu):
    """The stand-in carries every field benchmark.py:18-28 asserts, on the device."""
    from nf4_triton_dequantization_amd import Linear4bit

    lin = Linear4bit(512, 256, bias=None, compute_dtype=torch.float16, compress_statistics=True,
                     quant_type="nf4").to(gpu)
    assert lin.weight.device == gpu and lin.weight.quant_state.absmax.device == gpu
    out = _api().triton_dequantize_nf4(lin)
    assert out.shape == (256, 512) and out.dtype == torch.float16
    x = torch.randn(4, 512, device=gpu, dtype=torch.float16)
    y = lin(x)
    assert y.shape == (4, 256) and torch.isfinite(y).all()


def _double_rounding_scales(dt, count=64, seed=1):
    """Scales s and codes c where RNE16(fp32(NF4[c]*s)) != RNE16(exact NF4[c]*s): the
    reference rounds twice (fp32 product, then 16-bit cast); a fused multiply-convert
    would round once and differ exactly here."""
    rng = np.random.default_rng(seed)
    found_s, found_c = [], []
    lut = O.NF4_LUT.astype(np.float64)
    while len(found_s) < count:
        s = (rng.random(1 << 20) * 2.0 + 0.01).astype(np.float32)
        c = rng.integers(0, 16, 1 << 20)
        exact = lut[c] * s.astype(np.float64)
        f32 = exact.astype(np.float32)
        if dt == "f16":
            twice = f32.astype(np.float16).view(np.uint16)
            once = exact.astype(np.float16).view(np.uint16)
        else:
            twice = O.f32_to_bf16_bits(f32)
            u = exact.view(np.uint64)  # RNE of float64 to bf16 (8-bit mantissa)
            once = ((u + np.uint64(0x7FFFFFFFFFFF) + ((u >> np.uint64(48)) & np.uint64(1))) >> np.uint64(48))
            once = once.astype(np.uint16)
        hit = np.nonzero(twice != once)[0]
        found_s += s[hit].tolist()
        found_c += c[hit].tolist()
    return np.array(found_s[:count], np.float32), np.array(found_c[:count])


@pytest.mark.parametrize("dt", ["f16", "bf16"])
@pytest.mark.parametrize("n", [256, 200])  # 256: flat kernel, 200: chunk kernel
def test_double_rounding_and_signed_zero(coracle, gpu, dt, n):
    s, c = _double_rounding_scales(dt)
    bpr = (n + 63) // 64
    m = len(s) // bpr + 2
    scales = np.empty((m, bpr), np.float32)
    codes = np.empty((m, n), np.uint8)
    flat_s = np.concatenate([s, np.zeros(m * bpr - len(s), np.float32)])
    flat_c = np.concatenate([c, np.full(m * bpr - len(c), 3)])
    scales[:] = flat_s.reshape(m, bpr)
    scales[-1, :] = -0.0  # NF4 positive * -0 = -0 ; NF4 negative * -0 = +0
    scales[-2, :] = 0.0   # NF4 negative * +0 = -0
    for r in range(m):
        for b in range(bpr):
            codes[r, b * 64:(b + 1) * 64] = flat_c[r * bpr + b]
    codes[-2:, :] = np.arange(n) % 16
    if n % 2:
        codes = np.pad(codes, ((0, 0), (0, 1)))
    packed = ((codes[:, 0::2] << 4) | codes[:, 1::2]).astype(np.uint8).reshape(-1)
    want = coracle.dequant_single(packed, scales.reshape(-1), m, n, DT_CODE[dt])
    mod = make_module(packed, scales.reshape(-1), np.ones(1, np.float32), m, n, dt, gpu)
    assert_bits_equal(out_bits(_api().triton_dequantize_nf4(mod)), want, dt, f"double rounding {dt} n={n}")
    # the signed zeros are really there
    w = want[-2:].reshape(-1)
    assert (w == 0x8000).any() and (w == 0).any()


def test_host_quant_state_is_rejected(gpu):
    """absmax on the host with the packed weight on the GPU raises (no host pointer reaches a kernel)."""
    from nf4_triton_dequantization import triton_dequantize_nf4
    from nf4_triton_dequantization_amd import dequantize_nf4_many, nf4_linear

    packed, a1, a2 = O.make_inputs(64, 128, seed=2)
    mod = make_module(packed, a1, a2, 64, 128, "bf16", gpu)
    mod.weight.quant_state.absmax = mod.weight.quant_state.absmax.cpu()
    with pytest.raises(RuntimeError):
        triton_dequantize_nf4(mod)
    with pytest.raises(RuntimeError):
        dequantize_nf4_many([mod])
    with pytest.raises(RuntimeError):
        nf4_linear(torch.zeros(1, 128, dtype=torch.bfloat16, device=gpu), mod)


@pytest.mark.parametrize("dt", ["bf16", "f16", "f32"])
@pytest.mark.parametrize("ov", [{}, {"nb": 1000, "n2": 3}])
def test_multi_tile_waves(coracle, gpu, dt, ov):
    """Capped grids (1 and 2 workgroups per CU: every wave walks several tiles, odd and
    even counts), incl. the reference's wrapping absmax / nested absmax indices."""
    from nf4_triton_dequantization_amd import _lib

    m, n = 2048, 4160
    p, a1, a2, _ = O.golden_case_inputs(m, n, 91, ov)
    code = {"bf16": O.BF16, "f16": O.F16, "f32": O.F32}[dt]
    want = coracle.dequant_ref(p, a1, a2, m, n, code)
    tdt = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}[dt]
    q = torch.from_numpy(p).to(gpu)
    t1 = torch.from_numpy(a1).to(gpu)
    t2 = torch.from_numpy(a2).to(gpu)
    lcode = {"bf16": _lib.BF16, "f16": _lib.F16, "f32": _lib.F32}[dt]
    for cfg in ((4, 1, 1, 0), (4, 2, 1, 0)):
        out = torch.empty((m, n), dtype=tdt, device=gpu)
        c = _lib.LaunchCfg(*cfg)
        rc = _lib.lib().nf4_dequant_ref_cfg(q.data_ptr(), q.numel(), t1.data_ptr(), t1.numel(), t2.data_ptr(),
                                            t2.numel(), out.data_ptr(), lcode, m, n, ctypes.byref(c),
                                            torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        assert_bits_equal(out_bits(out), want, dt, f"cfg {cfg} {dt} {ov}")
