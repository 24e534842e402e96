"""Fused NF4 dequant-GEMM (``nf4_linear`` / ``nf4_gemm_ref``) vs a float64 oracle (``-m gpu``).

Oracle: W = the reference's dequantized weights from the C oracle (bit-exact
bf16/fp16, pinned to the reference fallback), X the same fp16/bf16 inputs, the
product in float64.  Tolerance (written here): fp32 accumulation of K terms
plus one final rounding to the output dtype,
    |y - ref| <= 2^-p |ref| + 2^-20 * sum_k |x_k w_k| + sub,   p = 8 (bf16), 10 (fp16),
where sub = half the output dtype's subnormal spacing (2^-25 fp16, 2^-134 bf16): an
output in the subnormal range rounds to an absolute, not a relative, grid (a drawn
fp16 case with y = 6.7e-7 is off by 9.7e-9 even when rounded from the exact sum).
"""
import numpy as np
import pytest
import torch

import nf4_oracle as O
from _helpers import make_module

pytestmark = pytest.mark.gpu


def _bits_to_f64(bits, dt):
    if dt == "f16":
        return bits.view(np.float16).astype(np.float64)
    return (bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def _tol(ref, mag, dt):
    p, sub = (8, 2.0 ** -134) if dt == "bf16" else (10, 2.0 ** -25)
    return 2.0 ** -p * np.abs(ref) + 2.0 ** -20 * mag + sub


def _check(y, x_bits, w_bits, dt):
    xf = _bits_to_f64(x_bits, dt)
    wf = _bits_to_f64(w_bits, dt)
    ref = xf @ wf.T
    mag = np.abs(xf) @ np.abs(wf).T
    tol = _tol(ref, mag, dt)
    yb = y.contiguous().view(torch.int16).cpu().numpy().view(np.uint16)
    got = _bits_to_f64(yb, dt).reshape(ref.shape)
    bad = np.abs(got - ref) > tol
    assert not bad.any(), f"{bad.sum()} of {bad.size} outside tolerance; worst {np.abs(got - ref).max():.3g}"


def _x_bits(M, K, dt, seed):
    x = O.normal_f32(seed, M * K, stream=9).reshape(M, K)
    t = torch.from_numpy(x).to(torch.float16 if dt == "f16" else torch.bfloat16)
    return t, t.view(torch.int16).numpy().view(np.uint16)


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("M,N,K", [(1, 64, 128), (3, 128, 512), (16, 256, 1024), (17, 192, 384), (32, 64, 4096),
                                   (1, 4096, 4096), (8, 1024, 4096), (4, 512, 11008), (2, 448, 14336),
                                   (24, 2048, 4096), (32, 4096, 1280), (17, 2112, 14336)])
def test_fused_gemm_vs_float64_oracle(coracle, gpu, dt, M, N, K):
    # the last three take the library's register-resident choice (16 < M <= 32,
    # N >= 2048, K % 256 == 0): two K slices, one slice with idle waves, seven slices
    from nf4_triton_dequantization_amd import nf4_linear

    packed, a1, a2 = O.make_inputs(N, K, seed=M * 7 + N + K, a2_kind="normal")
    W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16 if dt == "bf16" else O.F16)
    mod = make_module(packed, a1, a2, N, K, dt, gpu)
    xt, xb = _x_bits(M, K, dt, seed=M + K)
    y = nf4_linear(xt.to(gpu), mod)
    assert y.shape == (M, N) and y.dtype == xt.dtype
    _check(y, xb, W, dt)


def test_fused_matches_unfused_composite(gpu):
    """Same inputs through the fused kernel and through dequant + torch matmul."""
    from nf4_triton_dequantization import triton_dequantize_nf4
    from nf4_triton_dequantization_amd import nf4_linear

    packed, a1, a2 = O.make_inputs(1024, 4096, seed=5)
    mod = make_module(packed, a1, a2, 1024, 4096, "bf16", gpu)
    xt, _ = _x_bits(4, 4096, "bf16", seed=6)
    x = xt.to(gpu)
    y1 = nf4_linear(x, mod).float()
    y2 = (x.float() @ triton_dequantize_nf4(mod).float().t())
    assert torch.allclose(y1, y2, rtol=2 ** -7, atol=1e-2 * y2.abs().max().item())


def test_wrapping_absmax_and_leading_dims(coracle, gpu):
    """nb / n2 wrap (reference repeat semantics) and a [batch, seq, K] input."""
    from nf4_triton_dequantization_amd import nf4_linear

    N, K = 128, 256
    packed, a1, a2, _ = O.golden_case_inputs(N, K, 12, {"nb": 7, "n2": 3})
    W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16)
    mod = make_module(packed, a1, a2, N, K, "bf16", gpu)
    xt, xb = _x_bits(6, K, "bf16", seed=13)
    y = nf4_linear(xt.to(gpu).reshape(2, 3, K), mod)
    assert y.shape == (2, 3, N)
    _check(y.reshape(6, N), xb, W, "bf16")


@pytest.mark.parametrize("M", [1, 4, 12, 16])
def test_library_choice_falls_back_when_absmax_wraps_in_a_row(coracle, gpu, M):
    """At these M the library picks the decode GEMV (M = 1) or the persistent kernel
    (K-sliced above 8 rows), which need absmax without wrap inside a row; with a wrapping
    absmax (nb = 7, n2 = 3) it must fall back to the next choice -- single weight and
    grouped -- not fail."""
    from nf4_triton_dequantization_amd import nf4_linear, nf4_linear_grouped

    K = 4096
    Ns = (4096, 2048)
    mods, Ws = [], []
    for i, N in enumerate(Ns):
        packed, a1, a2, _ = O.golden_case_inputs(N, K, 40 + i, {"nb": 7 + i, "n2": 3})
        Ws.append(coracle.dequant_ref(packed, a1, a2, N, K, O.BF16))
        mods.append(make_module(packed, a1, a2, N, K, "bf16", gpu))
    xt, xb = _x_bits(M, K, "bf16", seed=M)
    x = xt.to(gpu)
    for mod, W in zip(mods, Ws):
        _check(nf4_linear(x, mod), xb, W, "bf16")
    for y, W in zip(nf4_linear_grouped(x, mods), Ws):
        _check(y, xb, W, "bf16")


def test_large_m_takes_composite_path(coracle, gpu):
    from nf4_triton_dequantization_amd import nf4_linear

    N, K, M = 256, 512, 80
    packed, a1, a2 = O.make_inputs(N, K, seed=21)
    W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16)
    mod = make_module(packed, a1, a2, N, K, "bf16", gpu)
    xt, xb = _x_bits(M, K, "bf16", seed=22)
    bias = torch.randn(N, device=gpu).to(torch.bfloat16)
    y = nf4_linear(xt.to(gpu), mod, bias=bias)
    y0 = nf4_linear(xt.to(gpu), mod)
    _check(y0, xb, W, "bf16")
    assert torch.allclose((y - y0).float(), bias.float().expand(M, N), atol=0.05)


def test_abi_rejects_non_fast_shapes(gpu):
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    F = 0x1000
    assert L.nf4_gemm_ref(F, 33, F, 64 * 64, F, 64, F, 1, F, _lib.BF16, 64, 128, None, 0, None) == _lib.ERR_SHAPE
    assert L.nf4_gemm_ref(F, 1, F, 32 * 64, F, 64, F, 1, F, _lib.BF16, 32, 128, None, 0, None) == _lib.ERR_SHAPE
    assert L.nf4_gemm_ref(F, 1, F, 64 * 48, F, 64, F, 1, F, _lib.BF16, 64, 96, None, 0, None) == _lib.ERR_SHAPE
    assert L.nf4_gemm_ref(F, 1, F, 64 * 64, F, 64, F, 1, F, _lib.F32, 64, 128, None, 0, None) == _lib.ERR_ARG
    import ctypes

    c = _lib.GemmCfg(_lib.GEMM_STREAM, 8, 4, 2, 1)
    need = L.nf4_gemm_workspace_bytes_cfg(1, 4096, 4096, ctypes.byref(c))
    assert need > 0
    # a K split without its workspace is an argument error, not a fault
    assert L.nf4_gemm_ref_cfg(F, 1, F, 4096 * 2048, F, 64, F, 1, F, _lib.BF16, 4096, 4096, None, 0,
                              ctypes.byref(c), None) == _lib.ERR_ARG


def test_workspace_reuse_across_shapes(coracle, gpu):
    """Calls of different N / split-K share one workspace; counters stay consistent."""
    from nf4_triton_dequantization_amd import nf4_linear

    for (M, N, K) in [(8, 1024, 4096), (1, 4096, 4096), (2, 64, 4096), (1, 4096, 4096), (4, 2048, 8192)] * 2:
        packed, a1, a2 = O.make_inputs(N, K, seed=N + K + M)
        W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16)
        mod = make_module(packed, a1, a2, N, K, "bf16", gpu)
        xt, xb = _x_bits(M, K, "bf16", seed=M + 1)
        _check(nf4_linear(xt.to(gpu), mod), xb, W, "bf16")


@pytest.mark.parametrize("M,N,K,cfg", [(8, 2560, 1280, (2, 4, 4, 4, 1)), (12, 384, 1280, (2, 4, 2, 4, 1)),
                                       (3, 256, 1792, (2, 8, 2, 6, 2)), (20, 128, 1792, (2, 8, 2, 5, 1))])
def test_streaming_kernel_empty_last_slices(coracle, gpu, M, N, K, cfg):
    """ksplit * ceil(chunks / ksplit) > chunks leaves the last slice(s) without chunks:
    they must add zero partials and take their tickets (found by tools/fuzz_gemm.py:
    the slice's range underflowed and its waves read past the staged x into NaN)."""
    import ctypes

    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    packed, a1, a2 = O.make_inputs(N, K, seed=N + K + M, a2_kind="normal")
    W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16)
    xt, xb = _x_bits(M, K, "bf16", seed=M + 3)
    mod_t = (torch.from_numpy(packed).to(gpu), torch.from_numpy(a1).to(gpu), torch.from_numpy(a2).to(gpu))
    y = torch.empty((M, N), dtype=torch.bfloat16, device=gpu)
    c = _lib.GemmCfg(*cfg)
    wsz = L.nf4_gemm_workspace_bytes_cfg(M, N, K, ctypes.byref(c))
    ws = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=gpu)
    rc = L.nf4_gemm_ref_cfg(xt.to(gpu).data_ptr(), M, mod_t[0].data_ptr(), mod_t[0].numel(), mod_t[1].data_ptr(),
                            mod_t[1].numel(), mod_t[2].data_ptr(), mod_t[2].numel(), y.data_ptr(), _lib.BF16, N, K,
                            ws.data_ptr(), wsz, ctypes.byref(c), torch.cuda.current_stream().cuda_stream)
    assert rc == 0, _lib.strerror(rc)
    assert L.nf4_gemm_check_workspace(ws.data_ptr(), wsz, torch.cuda.current_stream().cuda_stream) == 0
    _check(y, xb, W, "bf16")


@pytest.mark.parametrize("M,N,K", [(12, 1024, 4096), (16, 1024, 4096), (20, 28672, 4096), (24, 24576, 4096)])
def test_round4_default_rules(coracle, gpu, M, N, K):
    """The library defaults added in round 4: the register-resident kernel for
    1024-column launches at 8 < M <= 16, and its 16-wave whole-K form for the widest
    launches at 16 < M <= 24 (default_gemm_cfg / nonpersist_cfg)."""
    from nf4_triton_dequantization_amd import nf4_linear

    packed, a1, a2 = O.make_inputs(N, K, seed=5 * N + M, a2_kind="normal")
    W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16)
    mod = make_module(packed, a1, a2, N, K, "bf16", gpu)
    xt, xb = _x_bits(M, K, "bf16", seed=M + 19)
    _check(nf4_linear(xt.to(gpu), mod), xb, W, "bf16")


def test_check_gemm_workspaces_after_split_k(coracle, gpu):
    """nf4_linear's cached workspaces read clean after split-K launches (M = 16: the
    persistent kernel's K slices; M = 32: the register-resident kernel's two slices)."""
    from nf4_triton_dequantization_amd import check_gemm_workspaces, nf4_linear

    for (M, N, K) in [(16, 4096, 4096), (32, 2048, 4096), (12, 1024, 4096)]:
        packed, a1, a2 = O.make_inputs(N, K, seed=3 * N + M)
        W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16)
        mod = make_module(packed, a1, a2, N, K, "bf16", gpu)
        xt, xb = _x_bits(M, K, "bf16", seed=M + 7)
        _check(nf4_linear(xt.to(gpu), mod), xb, W, "bf16")
        assert check_gemm_workspaces() is None


def _gemm_cfg_call(L, _lib, xt, mod_t, y, dt_code, N, K, cfg):
    import ctypes

    packed, a1, a2 = mod_t
    M = xt.shape[0]
    wsz = L.nf4_gemm_workspace_bytes_cfg(M, N, K, ctypes.byref(cfg))
    ws = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=xt.device)
    rc = L.nf4_gemm_ref_cfg(xt.data_ptr(), M, packed.data_ptr(), packed.numel(), a1.data_ptr(), a1.numel(),
                            a2.data_ptr(), a2.numel(), y.data_ptr(), dt_code, N, K, ws.data_ptr(), wsz,
                            ctypes.byref(cfg), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return rc


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("M,N,K", [(1, 256, 4096), (5, 128, 2816), (16, 64, 1536), (32, 128, 2048),
                                   (1, 8192, 512), (3, 4160, 1280)])
def test_every_decomposition_agrees_with_oracle(coracle, gpu, dt, M, N, K):
    """Each kernel / waves / depth / strips / K-split combination the tuning ABI accepts."""
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    packed, a1, a2 = O.make_inputs(N, K, seed=N * 3 + K + M, a2_kind="normal")
    W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16 if dt == "bf16" else O.F16)
    t = (torch.from_numpy(packed).to(gpu), torch.from_numpy(a1).to(gpu), torch.from_numpy(a2).to(gpu))
    xt, xb = _x_bits(M, K, dt, seed=M * 5 + 1)
    x = xt.to(gpu)
    code = _lib.BF16 if dt == "bf16" else _lib.F16
    # the float64 oracle and its tolerance once; each config is compared on the GPU
    xf, wf = _bits_to_f64(xb, dt), _bits_to_f64(W, dt)
    ref = torch.from_numpy(xf @ wf.T).to(gpu)
    tol = torch.from_numpy(_tol(xf @ wf.T, np.abs(xf) @ np.abs(wf).T, dt)).to(gpu)
    y = torch.empty((M, N), dtype=x.dtype, device=gpu)
    ran = 0
    for kernel in (_lib.GEMM_PERSIST, _lib.GEMM_STREAM, _lib.GEMM_K128):
        for waves in (4, 8, 16):
            for depth in (1, 2, 4, 8):
                for strips in (1, 2, 4):  # K128: strips per wave
                    for ks in (1, 2, 3):
                        cfg = _lib.GemmCfg(kernel, waves, depth, ks, strips)
                        y.fill_(float("nan"))
                        rc = _gemm_cfg_call(L, _lib, x, t, y, code, N, K, cfg)
                        if rc == _lib.ERR_ARG:
                            continue
                        assert rc == 0, (kernel, waves, depth, strips, ks, rc)
                        bad = ((y.double() - ref).abs() > tol) | torch.isnan(y)
                        assert not bool(bad.any()), (kernel, waves, depth, strips, ks, int(bad.sum()))
                        ran += 1
    assert ran >= 12


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("M,K,kpw,spw", [(32, 4096, 2, 3), (32, 4096, 2, 9), (32, 4096, 2, 17), (17, 4096, 2, 3),
                                         (32, 2048, 1, 3), (24, 4096, 4, 3)])
def test_xr_multi_strip_workgroups(coracle, gpu, dt, M, K, kpw, spw):
    """The register-resident kernel with several 16-column strips per workgroup, at
    any CU count: N is sized from the device's CUs so that every workgroup walks >= spw
    strips (its ring refills, partial-tile reduction groups and cached weight
    descriptors all cross strip boundaries).  At two K slices (kpw = 2) the exchange
    form follows the strips per workgroup (launch_xr): spw = 3 takes the unrolled
    groups with GU = 4 (<= 8 strips), spw = 9 GU = 8 (<= 16 strips), both exchanging
    inside the strip loop, and spw = 17 the looped form (exchanges after the loop);
    kpw = 1 (four K slices) takes the ticket-and-poll hand-off."""
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    cus = torch.cuda.get_device_properties(gpu).multi_processor_count
    waves = 8
    ks = -(-(K // 128) // (waves * kpw))
    # the library's grid (xr_per_wg): one workgroup per CU, two for 128-deep chunks
    wg_per_slice = max(1, cus * (2 if kpw == 1 else 1) // ks)
    N = 16 * spw * wg_per_slice       # >= spw strips per workgroup
    N = -(-N // 64) * 64
    assert (N // 16) / wg_per_slice >= spw
    packed, a1, a2 = O.make_inputs(N, K, seed=N + K + M + kpw, a2_kind="normal")
    W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16 if dt == "bf16" else O.F16)
    t = (torch.from_numpy(packed).to(gpu), torch.from_numpy(a1).to(gpu), torch.from_numpy(a2).to(gpu))
    xt, xb = _x_bits(M, K, dt, seed=M * 3 + kpw)
    x = xt.to(gpu)
    y = torch.full((M, N), float("nan"), dtype=x.dtype, device=gpu)
    cfg = _lib.GemmCfg(_lib.GEMM_XR, waves, 2, ks, kpw)
    rc = _gemm_cfg_call(L, _lib, x, t, y, _lib.BF16 if dt == "bf16" else _lib.F16, N, K, cfg)
    assert rc == 0, rc
    assert not bool(torch.isnan(y).any())
    _check(y, xb, W, dt)


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("N,K", [(4096, 4096), (448, 14336), (64, 2048), (192, 16384), (14336, 4096)])
def test_gemv_every_decomposition(coracle, gpu, dt, N, K):
    """The decode GEMV (NF4DQ_GEMM_GEMV, M = 1): every waves / rows-per-group / grid form
    against the float64 oracle, outputs pre-filled with NaN (every row written)."""
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    packed, a1, a2 = O.make_inputs(N, K, seed=N * 5 + K, a2_kind="normal")
    W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16 if dt == "bf16" else O.F16)
    t = (torch.from_numpy(packed).to(gpu), torch.from_numpy(a1).to(gpu), torch.from_numpy(a2).to(gpu))
    xt, xb = _x_bits(1, K, dt, seed=K + 3)
    x = xt.to(gpu)
    code = _lib.BF16 if dt == "bf16" else _lib.F16
    xf, wf = _bits_to_f64(xb, dt), _bits_to_f64(W, dt)
    ref = torch.from_numpy(xf @ wf.T).to(gpu)
    tol = torch.from_numpy(_tol(xf @ wf.T, np.abs(xf) @ np.abs(wf).T, dt)).to(gpu)
    y = torch.empty((1, N), dtype=x.dtype, device=gpu)
    for waves in (8, 16):
        for rows in (1, 2, 4):
            for wgs in (0, 1, 2):  # workgroups per CU
                cfg = _lib.GemmCfg(_lib.GEMM_GEMV, waves, rows, 1, wgs)
                y.fill_(float("nan"))
                rc = _gemm_cfg_call(L, _lib, x, t, y, code, N, K, cfg)
                assert rc == 0, (waves, rows, wgs, rc)
                bad = ((y.double() - ref).abs() > tol) | torch.isnan(y)
                assert not bool(bad.any()), (waves, rows, wgs, int(bad.sum()))


def test_invalid_decompositions_rejected(gpu):
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    import ctypes

    F = 0x1000
    for cfg in [(_lib.GEMM_STREAM, 6, 4, 1, 1), (_lib.GEMM_STREAM, 8, 3, 1, 1), (_lib.GEMM_STREAM, 8, 4, 1, 3),
                (_lib.GEMM_STREAM, 4, 4, 1, 8), (_lib.GEMM_STREAM, 8, 4, 0, 1), (_lib.GEMM_STREAM, 8, 4, 99, 1),
                (_lib.GEMM_K128, 16, 2, 1, 1), (_lib.GEMM_K128, 8, 2, 1, 3), (9, 8, 4, 1, 1),
                (_lib.GEMM_GEMV, 8, 3, 1, 1), (_lib.GEMM_GEMV, 4, 1, 1, 1), (_lib.GEMM_GEMV, 16, 1, 2, 1),
                (_lib.GEMM_GEMV, 16, 1, 1, 3)]:
        c = _lib.GemmCfg(*cfg)
        assert L.nf4_gemm_ref_cfg(F, 1, F, 64 * 2048, F, 64 * 64, F, 16, F, _lib.BF16, 64, 4096, F, 1 << 30,
                                  ctypes.byref(c), None) == _lib.ERR_ARG, cfg
    # the streaming kernel needs K % 256 == 0
    c = _lib.GemmCfg(_lib.GEMM_STREAM, 8, 4, 1, 1)
    assert L.nf4_gemm_ref_cfg(F, 1, F, 64 * 64, F, 128, F, 1, F, _lib.BF16, 64, 128, F, 1 << 30,
                              ctypes.byref(c), None) == _lib.ERR_ARG


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("M,K,Ns", [(1, 4096, (4096, 1024, 1024)), (4, 2048, (512, 1536)),
                                    (3, 1280, (64, 128, 192, 256, 320, 384, 448, 512)), (16, 512, (1024, 64)),
                                    (24, 1280, (64, 128, 192, 256, 320)), (32, 4096, (4096, 1024, 1024)),
                                    (20, 384, (192, 64))])
def test_grouped_gemm_vs_float64_oracle(coracle, gpu, dt, M, K, Ns):
    """Weights sharing x in one launch: each output against its own float64 oracle."""
    from nf4_triton_dequantization_amd import nf4_linear_grouped

    mods, Ws = [], []
    for i, N in enumerate(Ns):
        packed, a1, a2 = O.make_inputs(N, K, seed=N + K + 11 * i, a2_kind="normal")
        Ws.append(coracle.dequant_ref(packed, a1, a2, N, K, O.BF16 if dt == "bf16" else O.F16))
        mods.append(make_module(packed, a1, a2, N, K, dt, gpu))
    xt, xb = _x_bits(M, K, dt, seed=M + 3)
    ys = nf4_linear_grouped(xt.to(gpu), mods)
    assert len(ys) == len(Ns)
    for y, W, N in zip(ys, Ws, Ns):
        assert y.shape == (M, N)
        _check(y, xb, W, dt)


def test_grouped_gemm_split_k_and_wrapping(coracle, gpu):
    """Grouped launch with a K split across workgroups and absmax that wraps (reference repeat)."""
    import ctypes

    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    M, K = 2, 1024
    Ns = (256, 128)
    specs = [(O.golden_case_inputs(256, K, 5, {"nb": 37, "n2": 5})[:3]), O.make_inputs(128, K, seed=9)]
    mats = (_lib.GemmMat * 2)()
    ys, keep, Ws = [], [], []
    for i, ((packed, a1, a2), N) in enumerate(zip(specs, Ns)):
        Ws.append(coracle.dequant_ref(packed, a1, a2, N, K, O.BF16))
        t = [torch.from_numpy(v).to(gpu) for v in (packed, a1, a2)]
        keep.append(t)
        y = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=gpu)
        ys.append(y)
        mats[i] = _lib.GemmMat(t[0].data_ptr(), t[0].numel(), t[1].data_ptr(), t[1].numel(), t[2].data_ptr(),
                               t[2].numel(), y.data_ptr(), N)
    xt, xb = _x_bits(M, K, "bf16", seed=21)
    x = xt.to(gpu)
    for ks in (1, 2, 3):
        cfg = _lib.GemmCfg(_lib.GEMM_STREAM, 8, 2, ks, 2)
        wsz = L.nf4_gemm_grouped_workspace_bytes(M, K, mats, 2, ctypes.byref(cfg))
        ws = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=gpu)
        rc = L.nf4_gemm_ref_grouped(x.data_ptr(), M, K, mats, 2, _lib.BF16, ws.data_ptr(), wsz, ctypes.byref(cfg),
                                    torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
        torch.cuda.synchronize()
        for y, W in zip(ys, Ws):
            _check(y, xb, W, "bf16")


@pytest.mark.parametrize("cfg", [(8, 2, 1, 1, 3), (4, 2, 2, 1, 3), (8, 4, 2, 1, 3), (16, 2, 2, 1, 3), (4, 4, 4, 1, 3),
                                 (8, 2, 4, 2, 16), (8, 2, 2, 2, 9), (8, 2, 4, 4, 16), (4, 2, 2, 4, 12),
                                 (16, 2, 4, 2, 5), (4, 2, 4, 8, 16)])
def test_persistent_grouped_gemm(coracle, gpu, cfg):
    """The persistent kernel over a grouped launch (several weights, several strip groups per
    workgroup), whole K or K slices (fp32 partials held in LDS, then the ticketed slab sum)."""
    import ctypes

    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    waves, depth, strips, ks, M = cfg
    K = 4096  # 16 chunks: every cfg above splits them into a multiple of its depth
    Ns = (4096, 1024, 2048)
    mats = (_lib.GemmMat * len(Ns))()
    ys, keep, Ws = [], [], []
    for i, N in enumerate(Ns):
        packed, a1, a2 = O.make_inputs(N, K, seed=7 * N + i, a2_kind="normal")
        Ws.append(coracle.dequant_ref(packed, a1, a2, N, K, O.BF16))
        t = [torch.from_numpy(v).to(gpu) for v in (packed, a1, a2)]
        keep.append(t)
        y = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=gpu)
        ys.append(y)
        mats[i] = _lib.GemmMat(t[0].data_ptr(), t[0].numel(), t[1].data_ptr(), t[1].numel(), t[2].data_ptr(),
                               t[2].numel(), y.data_ptr(), N)
    xt, xb = _x_bits(M, K, "bf16", seed=4)
    x = xt.to(gpu)
    c = _lib.GemmCfg(_lib.GEMM_PERSIST, waves, depth, ks, strips)
    wsz = L.nf4_gemm_grouped_workspace_bytes(M, K, mats, len(Ns), ctypes.byref(c))
    assert (wsz > 0) == (ks > 1)
    ws = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=gpu)
    for _ in range(2):  # the second call reuses the tickets the first left at 0
        for y in ys:
            y.fill_(float("nan"))
        rc = L.nf4_gemm_ref_grouped(x.data_ptr(), M, K, mats, len(Ns), _lib.BF16, ws.data_ptr() if wsz else None,
                                    wsz, ctypes.byref(c), torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
        torch.cuda.synchronize()
        for y, W in zip(ys, Ws):
            _check(y, xb, W, "bf16")
    if ks > 1:
        assert int(ws[:65536].view(torch.int32).abs().sum()) == 0  # tickets back at 0


@pytest.mark.parametrize("cfg", [(4, 2, 1, 1, 3), (8, 2, 2, 1, 16), (8, 2, 4, 2, 20), (4, 1, 2, 3, 32),
                                 (8, 4, 1, 4, 8), (8, 1, 4, 8, 32)])
@pytest.mark.parametrize("wrap", [False, True])
def test_k128_grouped_gemm(coracle, gpu, cfg, wrap):
    """The 128-deep kernel over ONE grouped launch (column groups numbered over all
    weights, K slices summed per group); `wrap` adds a weight whose absmax wraps inside
    a row, which turns the LDS scale table off for the whole launch."""
    import ctypes

    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    waves, depth, strips, ks, M = cfg
    K = 2048
    Ns = (1024, 256, 512) + ((128,) if wrap else ())
    mats = (_lib.GemmMat * len(Ns))()
    ys, keep, Ws = [], [], []
    for i, N in enumerate(Ns):
        if wrap and i == 3:
            packed, a1, a2 = O.golden_case_inputs(N, K, 5, {"nb": 37, "n2": 5})[:3]
        else:
            packed, a1, a2 = O.make_inputs(N, K, seed=3 * N + i, a2_kind="normal")
        Ws.append(coracle.dequant_ref(packed, a1, a2, N, K, O.BF16))
        t = [torch.from_numpy(v).to(gpu) for v in (packed, a1, a2)]
        keep.append(t)
        y = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=gpu)
        ys.append(y)
        mats[i] = _lib.GemmMat(t[0].data_ptr(), t[0].numel(), t[1].data_ptr(), t[1].numel(), t[2].data_ptr(),
                               t[2].numel(), y.data_ptr(), N)
    xt, xb = _x_bits(M, K, "bf16", seed=M + 40)
    x = xt.to(gpu)
    c = _lib.GemmCfg(_lib.GEMM_K128, waves, depth, ks, strips)
    wsz = L.nf4_gemm_grouped_workspace_bytes(M, K, mats, len(Ns), ctypes.byref(c))
    assert (wsz > 0) == (ks > 1)
    ws = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=gpu)
    for _ in range(2):  # the second call reuses the tickets the first left at 0
        for y in ys:
            y.fill_(float("nan"))
        rc = L.nf4_gemm_ref_grouped(x.data_ptr(), M, K, mats, len(Ns), _lib.BF16, ws.data_ptr() if wsz else None,
                                    wsz, ctypes.byref(c), torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
        torch.cuda.synchronize()
        for y, W in zip(ys, Ws):
            _check(y, xb, W, "bf16")
    if ks > 1:
        assert int(ws[:65536].view(torch.int32).abs().sum()) == 0  # tickets back at 0


def test_quantized_linears_grouped_fp16_bias(gpu):
    """NF4-quantize real-valued weights (our bitsandbytes-layout quantizer), then the grouped
    fused path with biases equals per-module dequant + matmul (same dequantized weights)."""
    from nf4_triton_dequantization import triton_dequantize_nf4
    from nf4_triton_dequantization_amd import nf4_linear, nf4_linear_grouped
    from nf4_triton_dequantization_amd.bnb_layout import Linear4bit

    torch.manual_seed(0)
    K = 2048
    mods, biases = [], []
    for N in (1024, 256, 256):
        lin = Linear4bit(K, N, bias=None, compute_dtype=torch.float16, weight=torch.randn(N, K) * 0.02)
        mods.append(lin.to(gpu))
        biases.append((torch.randn(N) * 0.1).to(torch.float16).to(gpu))
    x = (torch.randn(2, 3, K) * 0.5).to(torch.float16).to(gpu)
    ys = nf4_linear_grouped(x, mods, biases)
    for y, mod, b in zip(ys, mods, biases):
        W = triton_dequantize_nf4(mod).float()
        ref = x.float() @ W.t() + b.float()
        assert y.shape == (2, 3, W.shape[0]) and y.dtype == torch.float16
        assert torch.allclose(y.float(), ref, rtol=2 ** -9, atol=2e-3), (y.float() - ref).abs().max()
        y1 = nf4_linear(x, mod, bias=b)
        assert torch.allclose(y.float(), y1.float(), rtol=2 ** -9, atol=2e-3)


def test_host_activation_is_rejected(gpu):
    """x on the host and W on the GPU: RuntimeError (as `x @ W.t()`), never a host pointer in a kernel."""
    from nf4_triton_dequantization_amd import nf4_linear, nf4_linear_grouped

    packed, a1, a2 = O.make_inputs(128, 256, seed=3)
    mod = make_module(packed, a1, a2, 128, 256, "bf16", gpu)
    x = torch.randn(1, 256).to(torch.bfloat16)
    with pytest.raises(RuntimeError):
        nf4_linear(x, mod)
    with pytest.raises(RuntimeError):
        nf4_linear_grouped(x, [mod, mod])


@pytest.mark.parametrize("ks", [11, 12, 15])
def test_k128_slices_starting_past_the_end(coracle, gpu, ks):
    """K = 4096 (32 chunks of 128) with ksplit 11/12/15: ceil(32/ks) chunks per slice
    leaves the last slice(s) starting past the end; they must be empty (no wrapped
    scale-table count, no reads past absmax), single and grouped, table on."""
    import ctypes

    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    M, K, Ns = 20, 4096, (256, 128)
    mats = (_lib.GemmMat * len(Ns))()
    ys, keep, Ws = [], [], []
    for i, N in enumerate(Ns):
        packed, a1, a2 = O.make_inputs(N, K, seed=77 * N + ks, a2_kind="normal")
        Ws.append(coracle.dequant_ref(packed, a1, a2, N, K, O.BF16))
        t = [torch.from_numpy(v).to(gpu) for v in (packed, a1, a2)]
        keep.append(t)
        y = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=gpu)
        ys.append(y)
        mats[i] = _lib.GemmMat(t[0].data_ptr(), t[0].numel(), t[1].data_ptr(), t[1].numel(), t[2].data_ptr(),
                               t[2].numel(), y.data_ptr(), N)
    xt, xb = _x_bits(M, K, "bf16", seed=ks)
    x = xt.to(gpu)
    c = _lib.GemmCfg(_lib.GEMM_K128, 4, 1, ks, 1)
    wsz = L.nf4_gemm_grouped_workspace_bytes(M, K, mats, len(Ns), ctypes.byref(c))
    ws = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=gpu)
    rc = L.nf4_gemm_ref_grouped(x.data_ptr(), M, K, mats, len(Ns), _lib.BF16, ws.data_ptr(), wsz, ctypes.byref(c),
                                torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc
    torch.cuda.synchronize()
    for y, W in zip(ys, Ws):
        _check(y, xb, W, "bf16")
    # single-weight entry point with the same cfg
    y = torch.full((M, Ns[0]), float("nan"), dtype=torch.bfloat16, device=gpu)
    rc = _gemm_cfg_call(L, _lib, x, keep[0], y, _lib.BF16, Ns[0], K, c)
    assert rc == 0, rc
    torch.cuda.synchronize()
    _check(y, xb, Ws[0], "bf16")


def _xs_cfg(_lib, K, waves, kc):
    chunks = K // 128
    return _lib.GemmCfg(_lib.GEMM_XS, waves, kc, -(-chunks // kc), 1)


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("M,N,K", [(32, 1024, 4096), (17, 192, 1280), (24, 448, 384), (1, 64, 128), (9, 320, 2304),
                                   (32, 64, 11008), (30, 4160, 1024)])
def test_shared_activation_kernel_vs_oracle(coracle, gpu, dt, M, N, K):
    """NF4DQ_GEMM_XS, every (waves, chunks per slice) it accepts: full slices, a
    partial last slice (K/128 not a multiple), ksplit 1 (no slab) and > 1, a
    partial last strip group (N not a multiple of 16 x waves), M rows padded."""
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    packed, a1, a2 = O.make_inputs(N, K, seed=N + 3 * K + M, a2_kind="normal")
    W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16 if dt == "bf16" else O.F16)
    t = (torch.from_numpy(packed).to(gpu), torch.from_numpy(a1).to(gpu), torch.from_numpy(a2).to(gpu))
    xt, xb = _x_bits(M, K, dt, seed=M * 7 + 3)
    x = xt.to(gpu)
    code = _lib.BF16 if dt == "bf16" else _lib.F16
    y = torch.empty((M, N), dtype=x.dtype, device=gpu)
    ran = 0
    for waves in (4, 8):
        for kc in (2, 4, 8):
            cfg = _xs_cfg(_lib, K, waves, kc)
            for _ in range(2):  # twice: the tickets the first call left at 0 are reused
                y.fill_(float("nan"))
                rc = _gemm_cfg_call(L, _lib, x, t, y, code, N, K, cfg)
                assert rc == 0, (waves, kc, rc)
                _check(y, xb, W, dt)
            ran += 1
    assert ran == 6
    bad = _lib.GemmCfg(_lib.GEMM_XS, 8, 4, -(-(K // 128) // 4) + 1, 1)  # ksplit must be ceil(chunks / depth)
    assert _gemm_cfg_call(L, _lib, x, t, y, code, N, K, bad) == _lib.ERR_ARG


@pytest.mark.parametrize("wrap", [False, True])
def test_shared_activation_kernel_grouped(coracle, gpu, wrap):
    """One grouped launch of the shared-activation kernel (q/k/v-like); `wrap` adds a
    weight whose absmax / nested absmax wrap inside rows (the scale table gathers
    with the reference's modular indices, so no fallback is needed)."""
    import ctypes

    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    M, K = 32, 2048
    Ns = (1024, 256, 320) + ((128,) if wrap else ())
    mats = (_lib.GemmMat * len(Ns))()
    ys, keep, Ws = [], [], []
    for i, N in enumerate(Ns):
        if wrap and i == 3:
            packed, a1, a2 = O.golden_case_inputs(N, K, 5, {"nb": 37, "n2": 5})[:3]
        else:
            packed, a1, a2 = O.make_inputs(N, K, seed=5 * N + i, a2_kind="normal")
        Ws.append(coracle.dequant_ref(packed, a1, a2, N, K, O.BF16))
        tt = [torch.from_numpy(v).to(gpu) for v in (packed, a1, a2)]
        keep.append(tt)
        y = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=gpu)
        ys.append(y)
        mats[i] = _lib.GemmMat(tt[0].data_ptr(), tt[0].numel(), tt[1].data_ptr(), tt[1].numel(), tt[2].data_ptr(),
                               tt[2].numel(), y.data_ptr(), N)
    xt, xb = _x_bits(M, K, "bf16", seed=61)
    x = xt.to(gpu)
    for waves, kc in ((8, 4), (4, 8), (8, 2)):
        c = _xs_cfg(_lib, K, waves, kc)
        wsz = L.nf4_gemm_grouped_workspace_bytes(M, K, mats, len(Ns), ctypes.byref(c))
        ws = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=gpu)
        for y in ys:
            y.fill_(float("nan"))
        rc = L.nf4_gemm_ref_grouped(x.data_ptr(), M, K, mats, len(Ns), _lib.BF16, ws.data_ptr(), wsz,
                                    ctypes.byref(c), torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
        torch.cuda.synchronize()
        for y, W in zip(ys, Ws):
            _check(y, xb, W, "bf16")
        assert int(ws[:65536].view(torch.int32).abs().sum()) == 0  # tickets back at 0


def _xr_cfg(_lib, K, waves, depth, kpw):
    return _lib.GemmCfg(_lib.GEMM_XR, waves, depth, -(-(K // 128) // (waves * kpw)), kpw)


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("M,N,K", [(32, 1024, 4096), (17, 192, 1280), (24, 448, 384), (1, 64, 128), (9, 320, 2304),
                                   (32, 64, 11008), (16, 4160, 4096), (3, 2048, 4096)])
def test_register_resident_kernel_vs_oracle(coracle, gpu, dt, M, N, K):
    """NF4DQ_GEMM_XR, every (waves, depth, chunk depth) it accepts: one K slice
    (no slab: K = 4096 with 16 x 256-deep chunks) and several (the last one
    partial when K/128 is not a multiple), rows >= M padded, strips per workgroup
    from 1 up to the ring depth and beyond (partial last ring round)."""
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    packed, a1, a2 = O.make_inputs(N, K, seed=N + 5 * K + M, a2_kind="normal")
    W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16 if dt == "bf16" else O.F16)
    t = (torch.from_numpy(packed).to(gpu), torch.from_numpy(a1).to(gpu), torch.from_numpy(a2).to(gpu))
    xt, xb = _x_bits(M, K, dt, seed=M * 11 + 5)
    x = xt.to(gpu)
    code = _lib.BF16 if dt == "bf16" else _lib.F16
    y = torch.empty((M, N), dtype=x.dtype, device=gpu)
    ran = 0
    for waves in (8, 16):
        for depth in (2, 4):
            for kpw in (1, 2, 4):
                cfg = _xr_cfg(_lib, K, waves, depth, kpw)
                if ((M > 16 and kpw == 2 and depth == 4 and waves == 16) or (kpw == 2 and K % 256)
                        or (kpw == 4 and (waves != 8 or K % 512 or (M > 16 and depth == 4)))):
                    assert _gemm_cfg_call(L, _lib, x, t, y, code, N, K, cfg) == _lib.ERR_ARG
                    continue
                for _ in range(2):  # twice: the tickets the first call left at 0 are reused
                    y.fill_(float("nan"))
                    rc = _gemm_cfg_call(L, _lib, x, t, y, code, N, K, cfg)
                    assert rc == 0, (waves, depth, kpw, rc)
                    try:
                        _check(y, xb, W, dt)
                    except AssertionError as e:
                        raise AssertionError(f"cfg waves={waves} depth={depth} kpw={kpw}: {e}") from None
                ran += 1
    kpw4 = 0 if K % 512 else (1 if M > 16 else 2)  # 8 waves only; a 4-deep ring only up to 16 rows
    assert ran == (4 if K % 256 else 7 if M > 16 else 8) + kpw4
    bad = _lib.GemmCfg(_lib.GEMM_XR, 16, 2, -(-(K // 128) // 16) + 1, 1)  # ksplit must be ceil(chunks / 16)
    assert _gemm_cfg_call(L, _lib, x, t, y, code, N, K, bad) == _lib.ERR_ARG


@pytest.mark.parametrize("wrap", [False, True])
@pytest.mark.parametrize("M", [8, 32])
def test_register_resident_kernel_grouped(coracle, gpu, wrap, M):
    """One grouped launch of the register-resident kernel (q/k/v-like widths, an
    empty weight in the middle); `wrap` adds a weight whose absmax / nested
    absmax wrap inside rows (per-lane gathers with the reference's modular
    indices)."""
    import ctypes

    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    K = 2048
    Ns = (1024, 0, 256, 320) + ((128,) if wrap else ())
    mats = (_lib.GemmMat * len(Ns))()
    ys, keep, Ws = [], [], []
    for i, N in enumerate(Ns):
        if wrap and i == 4:
            packed, a1, a2 = O.golden_case_inputs(N, K, 5, {"nb": 37, "n2": 5})[:3]
        elif N == 0:
            packed, a1, a2 = (np.zeros(16, np.uint8), np.ones(4, np.uint8), np.ones(1, np.float32))
        else:
            packed, a1, a2 = O.make_inputs(N, K, seed=7 * N + i, a2_kind="normal")
        Ws.append(coracle.dequant_ref(packed, a1, a2, N, K, O.BF16) if N else None)
        tt = [torch.from_numpy(v).to(gpu) for v in (packed, a1, a2)]
        keep.append(tt)
        y = torch.full((M, max(N, 1)), float("nan"), dtype=torch.bfloat16, device=gpu)
        ys.append(y)
        mats[i] = _lib.GemmMat(tt[0].data_ptr(), N * K // 2, tt[1].data_ptr(), tt[1].numel(), tt[2].data_ptr(),
                               tt[2].numel(), y.data_ptr(), N)
    xt, xb = _x_bits(M, K, "bf16", seed=67 + M)
    x = xt.to(gpu)
    for waves, depth, kpw in ((16, 4, 1), (16, 2, 2), (8, 2, 1), (8, 4, 1), (8, 2, 4)):
        c = _xr_cfg(_lib, K, waves, depth, kpw)
        wsz = L.nf4_gemm_grouped_workspace_bytes(M, K, mats, len(Ns), ctypes.byref(c))
        ws = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=gpu)
        for y in ys:
            y.fill_(float("nan"))
        rc = L.nf4_gemm_ref_grouped(x.data_ptr(), M, K, mats, len(Ns), _lib.BF16, ws.data_ptr(), wsz,
                                    ctypes.byref(c), torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
        torch.cuda.synchronize()
        for y, W in zip(ys, Ws):
            if W is not None:
                _check(y, xb, W, "bf16")
        assert int(ws[:65536].view(torch.int32).abs().sum()) == 0  # tickets back at 0


try:
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st

    @st.composite
    def _gemm_cases(draw):
        M = draw(st.integers(1, 32))
        N = 64 * draw(st.integers(1, 48))
        K = draw(st.sampled_from([128, 256, 384, 512, 1024, 1280, 2048, 2304, 4096, 4352]))
        wrap = draw(st.booleans())
        dt = draw(st.sampled_from(["bf16", "f16"]))
        seed = draw(st.integers(0, 2 ** 31 - 1))
        return M, N, K, wrap, dt, seed

    @settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                     HealthCheck.function_scoped_fixture])
    @given(_gemm_cases())
    def test_library_choice_property(coracle, gpu, case):
        """Drawn shapes through nf4_linear (the library's decomposition choice for each M,
        N, K -- every kernel family is reachable), with and without absmax / nested
        absmax wrapping inside rows, against the float64 oracle."""
        from nf4_triton_dequantization_amd import nf4_linear

        M, N, K, wrap, dt, seed = case
        if wrap:
            packed, a1, a2, _ = O.golden_case_inputs(N, K, seed % 100000, {"nb": 37, "n2": 5, "a2_kind": "normal"})
        else:
            packed, a1, a2 = O.make_inputs(N, K, seed=seed % 100000, a2_kind="normal")
        W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16 if dt == "bf16" else O.F16)
        mod = make_module(packed, a1, a2, N, K, dt, gpu)
        xt, xb = _x_bits(M, K, dt, seed=seed % 1000 + 1)
        y = nf4_linear(xt.to(gpu), mod)
        assert y.shape == (M, N)
        _check(y, xb, W, dt)
    @st.composite
    def _group_cases(draw):
        M = draw(st.integers(1, 32))
        K = draw(st.sampled_from([128, 384, 1024, 2048, 4096]))
        Ns = draw(st.lists(st.integers(1, 40).map(lambda v: 64 * v), min_size=2, max_size=4))
        wraps = draw(st.lists(st.booleans(), min_size=len(Ns), max_size=len(Ns)))
        seed = draw(st.integers(0, 10 ** 6))
        return M, K, Ns, wraps, seed

    @settings(max_examples=30, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                     HealthCheck.function_scoped_fixture])
    @given(_group_cases())
    def test_grouped_library_choice_property(coracle, gpu, case):
        """Drawn weight groups (2-4 weights sharing x, some with absmax wrapping inside a
        row) through nf4_linear_grouped -- one launch, the library's choice -- each output
        against the float64 oracle."""
        from nf4_triton_dequantization_amd import nf4_linear_grouped

        M, K, Ns, wraps, seed = case
        mods, Ws = [], []
        for i, (N, wrap) in enumerate(zip(Ns, wraps)):
            if wrap:
                packed, a1, a2, _ = O.golden_case_inputs(N, K, seed + i, {"nb": 11 + i, "n2": 3, "a2_kind": "normal"})
            else:
                packed, a1, a2 = O.make_inputs(N, K, seed=seed + i, a2_kind="normal")
            Ws.append(coracle.dequant_ref(packed, a1, a2, N, K, O.BF16))
            mods.append(make_module(packed, a1, a2, N, K, "bf16", gpu))
        xt, xb = _x_bits(M, K, "bf16", seed=seed % 997 + 3)
        ys = nf4_linear_grouped(xt.to(gpu), mods)
        for y, W, N in zip(ys, Ws, Ns):
            assert y.shape == (M, N)
            _check(y, xb, W, "bf16")
except ImportError:  # hypothesis is part of the test environment; keep the module importable without it
    pass


def test_retired_balanced_kernel_is_rejected(gpu):
    """NF4DQ_GEMM_SK (the stream-K kernel, never the library's choice) was removed in
    round 6: a cfg naming it is rejected with ERR_ARG before any device work, at shapes
    it used to run (14336x4096 at M = 1, a grouped launch) as well as the others."""
    import ctypes

    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    F = 0x1000
    c = _lib.GemmCfg(_lib.GEMM_SK, 8, 0, 1, 0)
    for (M, N, K) in [(1, 14336, 4096), (4, 4096, 4096), (1, 64, 2048), (9, 4096, 4096), (1, 4096, 1152)]:
        rc = L.nf4_gemm_ref_cfg(F, M, F, N * K // 2, F, N * K // 64, F, 16, F, _lib.BF16, N, K, F, 1 << 30,
                                ctypes.byref(c), None)
        assert rc == _lib.ERR_ARG, (M, N, K, rc)
    arr = (_lib.GemmMat * 1)()
    arr[0] = _lib.GemmMat(F, 14336 * 2048, F, 14336 * 64, F, 16, F, 14336)
    assert L.nf4_gemm_grouped_workspace_bytes(1, 4096, arr, 1, ctypes.byref(c)) == 0
    rc = L.nf4_gemm_ref_grouped(F, 1, 4096, arr, 1, _lib.BF16, F, 1 << 30, ctypes.byref(c), None)
    assert rc == _lib.ERR_ARG, rc


def _splitk3_cfg(L, _lib, x, t, y, N, K):
    """A persistent-kernel configuration with more than two K slices (ticket + poll
    hand-off, splitk_reduce; two slices would take the exchange) that the library
    accepts for this shape."""
    for ks in (4, 3, 8):
        for waves in (4, 8, 16):
            for depth in (1, 2, 4, 8):
                for strips in (1, 2, 4):
                    cfg = _lib.GemmCfg(_lib.GEMM_PERSIST, waves, depth, ks, strips)
                    if _gemm_cfg_call(L, _lib, x, t, y, _lib.BF16, N, K, cfg) == 0:
                        return cfg
    raise AssertionError("no persistent configuration with > 2 K slices accepted")


def test_splitk_error_word_is_reported_and_poisons_later_calls(coracle, gpu):
    """the split-K error path.  A set error word (what a reducer that gave
    up waiting leaves) is reported by nf4_gemm_check_workspace as ERR_SPLITK_TIMEOUT and
    the workspace comes back zeroed; while it is set, every split-K reducer writes NaN
    instead of a sum (a timed-out slice's late store could otherwise pass for a
    written partial in a later call); after the check the next call is exact again."""
    import ctypes

    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    M, N, K = 4, 256, 4096
    packed, a1, a2 = O.make_inputs(N, K, seed=4242, a2_kind="normal")
    W = coracle.dequant_ref(packed, a1, a2, N, K, O.BF16)
    t = (torch.from_numpy(packed).to(gpu), torch.from_numpy(a1).to(gpu), torch.from_numpy(a2).to(gpu))
    xt, xb = _x_bits(M, K, "bf16", seed=31)
    x = xt.to(gpu)
    y = torch.empty((M, N), dtype=torch.bfloat16, device=gpu)
    cfg = _splitk3_cfg(L, _lib, x, t, y, N, K)
    wsz = L.nf4_gemm_workspace_bytes_cfg(M, N, K, ctypes.byref(cfg))
    assert wsz >= 65536 + 4
    ws = torch.zeros(wsz, dtype=torch.uint8, device=gpu)
    sp = torch.cuda.current_stream().cuda_stream

    def run():
        y.fill_(0.0)
        rc = L.nf4_gemm_ref_cfg(x.data_ptr(), M, t[0].data_ptr(), t[0].numel(), t[1].data_ptr(), t[1].numel(),
                                t[2].data_ptr(), t[2].numel(), y.data_ptr(), _lib.BF16, N, K, ws.data_ptr(), wsz,
                                ctypes.byref(cfg), sp)
        torch.cuda.synchronize()
        assert rc == 0, _lib.strerror(rc)

    run()
    _check(y, xb, W, "bf16")
    assert L.nf4_gemm_check_workspace(ws.data_ptr(), wsz, sp) == _lib.OK
    # 1. reported, and the workspace is re-zeroed
    ws[65536] = 1
    assert L.nf4_gemm_check_workspace(ws.data_ptr(), wsz, sp) == _lib.ERR_SPLITK_TIMEOUT
    assert int(ws.count_nonzero()) == 0
    assert L.nf4_gemm_check_workspace(ws.data_ptr(), wsz, sp) == _lib.OK
    # 2. a set word poisons the next calls: NaN, never a sum of possibly stale partials
    ws[65536] = 1
    run()
    assert bool(torch.isnan(y.float()).all())
    run()
    assert bool(torch.isnan(y.float()).all())
    assert L.nf4_gemm_check_workspace(ws.data_ptr(), wsz, sp) == _lib.ERR_SPLITK_TIMEOUT
    run()
    _check(y, xb, W, "bf16")
    assert L.nf4_gemm_check_workspace(ws.data_ptr(), wsz, sp) == _lib.OK


def test_check_gemm_workspaces_raises_on_a_set_error_word(coracle, gpu):
    """check_gemm_workspaces() raises RuntimeError naming the stream when a cached
    workspace's error word is set, and is clean on the next check (the library zeroed it)."""
    from nf4_triton_dequantization_amd import check_gemm_workspaces, kernel, nf4_linear

    M, N, K = 16, 4096, 4096  # the persistent kernel's K slices: a cached workspace
    packed, a1, a2 = O.make_inputs(N, K, seed=77)
    mod = make_module(packed, a1, a2, N, K, "bf16", gpu)
    xt, _ = _x_bits(M, K, "bf16", seed=3)
    nf4_linear(xt.to(gpu), mod)
    torch.cuda.synchronize()
    key = (gpu.index if gpu.index is not None else 0, torch.cuda.current_stream(gpu).cuda_stream)
    assert key in kernel._GEMM_WS
    ws, _stream = kernel._GEMM_WS[key]
    assert check_gemm_workspaces() is None
    ws[65536] = 1
    with pytest.raises(RuntimeError, match="split-K"):
        check_gemm_workspaces()
    assert check_gemm_workspaces() is None


def test_release_gemm_workspaces_reports_a_pending_error(coracle, gpu):
    """release_gemm_workspaces() reads each cached workspace's sticky error
    word before forgetting it, so a split-K timeout since the last check is raised, not
    lost -- and the cache is cleared either way."""
    from nf4_triton_dequantization_amd import kernel, nf4_linear, release_gemm_workspaces

    M, N, K = 16, 4096, 4096
    packed, a1, a2 = O.make_inputs(N, K, seed=79)
    mod = make_module(packed, a1, a2, N, K, "bf16", gpu)
    xt, _ = _x_bits(M, K, "bf16", seed=5)
    nf4_linear(xt.to(gpu), mod)
    torch.cuda.synchronize()
    key = (gpu.index if gpu.index is not None else 0, torch.cuda.current_stream(gpu).cuda_stream)
    ws, _stream = kernel._GEMM_WS[key]
    ws[65536] = 1  # the error word a reducer sets when its poll gives up
    with pytest.raises(RuntimeError, match="split-K"):
        release_gemm_workspaces()
    assert not kernel._GEMM_WS


def test_release_gemm_workspaces_empties_the_cache(gpu):
    """release_gemm_workspaces() synchronises the cached workspaces' streams and forgets
    them (for callers that destroy their own external streams); nf4_linear then builds a
    fresh one on its next call."""
    from nf4_triton_dequantization_amd import kernel, nf4_linear, release_gemm_workspaces

    M, N, K = 16, 4096, 4096
    packed, a1, a2 = O.make_inputs(N, K, seed=78)
    mod = make_module(packed, a1, a2, N, K, "bf16", gpu)
    xt, _ = _x_bits(M, K, "bf16", seed=4)
    y0 = nf4_linear(xt.to(gpu), mod)
    assert kernel._GEMM_WS
    release_gemm_workspaces()
    assert not kernel._GEMM_WS
    y1 = nf4_linear(xt.to(gpu), mod)
    torch.cuda.synchronize()
    assert kernel._GEMM_WS and torch.equal(y0.view(torch.int16), y1.view(torch.int16))
