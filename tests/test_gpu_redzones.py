"""Guard-band checks of every C-ABI entry point on the GPU (``-m gpu``).

SURVEY §5 asks for sanitizer coverage; GPU AddressSanitizer is not available on
this pool, so this is the device-side stand-in: every buffer an entry point is
handed -- inputs, outputs, the GEMM workspace -- is carved out of a larger
allocation with 64 KiB guard bands of a fixed byte pattern on both sides.  After
each call: both bands of every buffer intact (no write outside a buffer), the
inputs unchanged (no write into an input), the output equal to the oracle, and
the split-K ticket counters, error word and slab entries back at zero
(nf4_gemm_check_workspace returns OK).  Shapes take ragged tails (partial
tiles, partial 64-blocks, odd n, single rows, wrapping / truncated statistics,
strips not filling a workgroup), where range handling matters.
(The host path has its own ASan/UBSan run: tests/test_cpu_sanitizers.py.)
"""
import ctypes

import numpy as np
import pytest
import torch

import nf4_oracle as O
from _helpers import DT_CODE, assert_bits_equal, out_bits, torch_dtype

pytestmark = pytest.mark.gpu

GUARD = 64 * 1024
PAT = 0xA5
COUNTER_BYTES = 64 * 1024  # split-K tickets at the head of the GEMM workspace (nf4_gemm.hip kCounterBytes);
# the error word and 252 spare bytes follow (kHeaderBytes = 64 KiB + 256), then the slab


class Guarded:
    """``nbytes`` usable bytes between two guard bands (offset 64 KiB: 256-B aligned)."""

    def __init__(self, nbytes, device, fill=PAT):
        self.n = int(nbytes)
        self.buf = torch.full((2 * GUARD + max(self.n, 1),), PAT, dtype=torch.uint8, device=device)
        if fill != PAT:
            self.buf[GUARD:GUARD + self.n].fill_(fill)

    @classmethod
    def of(cls, arr: np.ndarray, device):
        g = cls(arr.nbytes, device)
        if arr.nbytes:
            g.buf[GUARD:GUARD + g.n].copy_(torch.from_numpy(np.ascontiguousarray(arr).reshape(-1).view(np.uint8)))
        return g

    def body(self, dtype=torch.uint8):
        return self.buf[GUARD:GUARD + self.n].view(dtype)

    def ptr(self):
        return self.buf.data_ptr() + GUARD

    def bands_intact(self):
        return bool((self.buf[:GUARD] == PAT).all()) and bool((self.buf[GUARD + self.n:] == PAT).all())


def _inputs_intact(pairs):
    for g, arr in pairs:
        assert g.bands_intact(), "guard band of an input overwritten"
        got = g.body().cpu().numpy()
        assert np.array_equal(got, np.ascontiguousarray(arr).reshape(-1).view(np.uint8)), "input modified"


def _stream():
    return torch.cuda.current_stream().cuda_stream


ELT = {"f16": 2, "bf16": 2, "f32": 4}
REF_SHAPES = [(1, 1, {}), (3, 70, {}), (17, 130, {"nb": 5, "n2": 2}), (5, 4097, {}), (64, 4096, {"n2": 3}),
              (333, 777, {"nb": 1000}), (1024, 1024, {}), (2, 64, {"stride": 40})]


@pytest.mark.parametrize("dt", ["bf16", "f16", "f32"])
def test_dequant_ref_and_single(coracle, gpu, dt):
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    for i, (m, n, ov) in enumerate(REF_SHAPES):
        p, a1, a2, single = O.golden_case_inputs(m, n, 100 + i, dict({"stride": (n + 1) // 2}, **ov, single=1))
        gp, ga1, ga2, gs = (Guarded.of(v, gpu) for v in (p, a1, a2, single))
        out = Guarded(m * n * ELT[dt], gpu, fill=0x5A)
        rc = L.nf4_dequant_ref(gp.ptr(), p.size, ga1.ptr(), a1.size, ga2.ptr(), a2.size, out.ptr(), DT_CODE[dt],
                               m, n, _stream())
        torch.cuda.synchronize()
        assert rc == 0, _lib.strerror(rc)
        assert out.bands_intact(), f"write outside the output, {m}x{n}"
        assert_bits_equal(out_bits(out.body(torch_dtype(dt)).view(m, n)), coracle.dequant_ref(p, a1, a2, m, n, DT_CODE[dt]),
                          dt, f"ref {m}x{n}")
        out2 = Guarded(m * n * ELT[dt], gpu, fill=0x5A)
        rc = L.nf4_dequant_single(gp.ptr(), p.size, gs.ptr(), single.size, out2.ptr(), DT_CODE[dt], m, n,
                                  _stream())
        torch.cuda.synchronize()
        assert rc == 0, _lib.strerror(rc)
        assert out2.bands_intact(), f"write outside the output (single), {m}x{n}"
        assert_bits_equal(out_bits(out2.body(torch_dtype(dt)).view(m, n)), coracle.dequant_single(p, single, m, n, DT_CODE[dt]),
                          dt, f"single {m}x{n}")
        _inputs_intact([(gp, p), (ga1, a1), (ga2, a2), (gs, single)])


def test_batched(coracle, gpu):
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    descs, keep, want = [], [], []
    for i, (m, n, ov) in enumerate(REF_SHAPES):
        p, a1, a2, _ = O.golden_case_inputs(m, n, 200 + i, dict({"stride": (n + 1) // 2}, **ov))
        gp, ga1, ga2 = (Guarded.of(v, gpu) for v in (p, a1, a2))
        out = Guarded(m * n * 2, gpu, fill=0x5A)
        descs.append(_lib.MatrixDesc(gp.ptr(), p.size, ga1.ptr(), a1.size, ga2.ptr(), a2.size, out.ptr(), m, n))
        keep.append((gp, ga1, ga2, out, (p, a1, a2)))
        want.append(coracle.dequant_ref(p, a1, a2, m, n, O.BF16))
    arr = (_lib.MatrixDesc * len(descs))(*descs)
    rc = L.nf4_dequant_ref_batched(arr, len(descs), _lib.BF16, _stream())
    torch.cuda.synchronize()
    assert rc == 0, _lib.strerror(rc)
    for (gp, ga1, ga2, out, (p, a1, a2)), w, (m, n, _) in zip(keep, want, REF_SHAPES):
        assert out.bands_intact(), f"write outside the output, {m}x{n}"
        assert_bits_equal(out_bits(out.body(torch.bfloat16).view(m, n)), w, "bf16", f"batched {m}x{n}")
        _inputs_intact([(gp, p), (ga1, a1), (ga2, a2)])


@pytest.mark.parametrize("bs", [64, 256, 4096])
def test_bnb(coracle, gpu, bs):
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    for numel in (1, 63, 65, bs * 3 + 1, 64 * 256 * 2 + 130):
        nblk = (numel + bs - 1) // bs
        p = O.splitmix64_bytes(numel, (numel + 1) // 2, stream=1)
        a1 = O.splitmix64_bytes(numel, nblk, stream=2)
        code2 = O.normal_f32(numel, 256, stream=5)
        a2 = O.uniform_f32(numel, (nblk + 255) // 256, 1e-3, 1e-1, stream=3)
        am = O.uniform_f32(numel, nblk, 1e-3, 1.0, stream=4)
        gp, ga1, gc, ga2, gam = (Guarded.of(v, gpu) for v in (p, a1, code2, a2, am))
        out = Guarded(numel * 2, gpu, fill=0x5A)
        rc = L.nf4_dequant_bnb(gp.ptr(), ga1.ptr(), a1.size, gc.ptr(), ga2.ptr(), a2.size, 0.25, out.ptr(), _lib.BF16,
                               numel, bs, 256, _stream())
        torch.cuda.synchronize()
        assert rc == 0, _lib.strerror(rc)
        assert out.bands_intact(), f"write outside the output, numel {numel}"
        assert_bits_equal(out_bits(out.body(torch.bfloat16)),
                          coracle.dequant_bnb(p, a1, code2, a2, 0.25, numel, O.BF16, bs, 256), "bf16", f"bnb {numel}")
        out2 = Guarded(numel * 2, gpu, fill=0x5A)
        rc = L.nf4_dequant_bnb_single(gp.ptr(), gam.ptr(), am.size, out2.ptr(), _lib.BF16, numel, bs, _stream())
        torch.cuda.synchronize()
        assert rc == 0, _lib.strerror(rc)
        assert out2.bands_intact(), f"write outside the output (single), numel {numel}"
        assert_bits_equal(out_bits(out2.body(torch.bfloat16)), coracle.dequant_bnb_single(p, am, numel, O.BF16, bs),
                          "bf16", f"bnb single {numel}")
        _inputs_intact([(gp, p), (ga1, a1), (gc, code2), (ga2, a2), (gam, am)])


def _gemm_cfgs(K):
    from nf4_triton_dequantization_amd import _lib

    chunks = K // 128
    for kernel in (_lib.GEMM_PERSIST, _lib.GEMM_STREAM, _lib.GEMM_K128):
        for waves in (4, 8, 16):
            for depth in (1, 2, 4):
                for strips in (1, 2, 4):
                    for ks in (1, 2, 3):
                        yield _lib.GemmCfg(kernel, waves, depth, ks, strips)
    for waves in (4, 8):
        for kc in (2, 4, 8):
            yield _lib.GemmCfg(_lib.GEMM_XS, waves, kc, -(-chunks // kc), 1)
    for waves in (8, 16):
        for depth in (2, 4):
            for kpw in (1, 2, 4):
                yield _lib.GemmCfg(_lib.GEMM_XR, waves, depth, -(-chunks // (waves * kpw)), kpw)


def _gemm_ref(W_bits, x_bits):
    xf = (x_bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    wf = (W_bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    ref = xf @ wf.T
    tol = 2.0 ** -8 * np.abs(ref) + 2.0 ** -20 * (np.abs(xf) @ np.abs(wf).T)
    return ref, tol


@pytest.mark.parametrize("M,N,K", [(3, 192, 384), (17, 4160, 1280), (32, 2112, 4096), (1, 64, 2048),
                                   (5, 4160, 1280), (2, 1024, 4096)])
def test_gemm_every_decomposition(coracle, gpu, M, N, K):
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    p, a1, a2 = O.make_inputs(N, K, seed=M + N + K, a2_kind="normal")
    W = coracle.dequant_ref(p, a1, a2, N, K, O.BF16)
    x = torch.from_numpy(O.normal_f32(M + 1, M * K, stream=9).reshape(M, K)).to(torch.bfloat16)
    xb = x.view(torch.int16).numpy().view(np.uint16)
    ref, tol = _gemm_ref(W, xb)
    ref_t, tol_t = torch.from_numpy(ref).to(gpu), torch.from_numpy(tol).to(gpu)
    gp, ga1, ga2, gx = (Guarded.of(v, gpu) for v in (p, a1, a2, xb))
    ran = 0
    for cfg in _gemm_cfgs(K):
        wsz = L.nf4_gemm_workspace_bytes_cfg(M, N, K, ctypes.byref(cfg))
        ws = Guarded(wsz, gpu, fill=0)
        y = Guarded(M * N * 2, gpu, fill=0x5A)
        rc = L.nf4_gemm_ref_cfg(gx.ptr(), M, gp.ptr(), p.size, ga1.ptr(), a1.size, ga2.ptr(), a2.size, y.ptr(),
                                _lib.BF16, N, K, ws.ptr() if wsz else None, wsz, ctypes.byref(cfg), _stream())
        torch.cuda.synchronize()
        if rc == _lib.ERR_ARG:
            continue
        what = (cfg.kernel, cfg.waves, cfg.depth, cfg.ksplit, cfg.strips)
        assert rc == 0, (what, _lib.strerror(rc))
        assert y.bands_intact(), f"write outside y, cfg {what}"
        assert ws.bands_intact(), f"write outside the workspace, cfg {what}"
        # the split-K error word: no reducer gave up
        assert L.nf4_gemm_check_workspace(ws.ptr() if wsz else None, wsz, _stream()) == 0, what
        if wsz:
            # tickets back at 0 and every split-K slab entry read and cleared (empty) again
            assert int(ws.body()[:min(COUNTER_BYTES, wsz)].count_nonzero()) == 0, f"tickets not reset, cfg {what}"
            assert int(ws.body().count_nonzero()) == 0, f"slab entries not cleared, cfg {what}"
        bad = (y.body(torch.bfloat16).view(M, N).double() - ref_t).abs() > tol_t
        assert not bool(bad.any()), (what, int(bad.sum()))
        ran += 1
    _inputs_intact([(gp, p), (ga1, a1), (ga2, a2), (gx, xb)])
    assert ran >= 8, ran


def test_gemm_grouped(coracle, gpu):
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    M, K = 5, 1280
    Ns = (64, 4160, 192)
    x = torch.from_numpy(O.normal_f32(7, M * K, stream=9).reshape(M, K)).to(torch.bfloat16)
    xb = x.view(torch.int16).numpy().view(np.uint16)
    gx = Guarded.of(xb, gpu)
    mats = (_lib.GemmMat * len(Ns))()
    keep = []
    for i, N in enumerate(Ns):
        p, a1, a2 = O.make_inputs(N, K, seed=300 + i, a2_kind="normal")
        gp, ga1, ga2 = (Guarded.of(v, gpu) for v in (p, a1, a2))
        y = Guarded(M * N * 2, gpu, fill=0x5A)
        mats[i] = _lib.GemmMat(gp.ptr(), p.size, ga1.ptr(), a1.size, ga2.ptr(), a2.size, y.ptr(), N)
        keep.append((N, gp, ga1, ga2, y, (p, a1, a2)))
    wsz = L.nf4_gemm_grouped_workspace_bytes(M, K, mats, len(Ns), None)
    ws = Guarded(wsz, gpu, fill=0)
    rc = L.nf4_gemm_ref_grouped(gx.ptr(), M, K, mats, len(Ns), _lib.BF16, ws.ptr() if wsz else None, wsz, None,
                                _stream())
    torch.cuda.synchronize()
    assert rc == 0, _lib.strerror(rc)
    assert ws.bands_intact()
    assert L.nf4_gemm_check_workspace(ws.ptr() if wsz else None, wsz, _stream()) == 0
    if wsz:
        assert int(ws.body().count_nonzero()) == 0  # tickets and slab entries back at 0
    for N, gp, ga1, ga2, y, (p, a1, a2) in keep:
        assert y.bands_intact(), f"write outside y of the {N}-column weight"
        ref, tol = _gemm_ref(coracle.dequant_ref(p, a1, a2, N, K, O.BF16), xb)
        got = y.body(torch.bfloat16).view(M, N).double().cpu().numpy()
        assert not (np.abs(got - ref) > tol).any(), N
        _inputs_intact([(gp, p), (ga1, a1), (ga2, a2)])
    _inputs_intact([(gx, xb)])
