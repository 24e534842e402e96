"""The library's host path (``nf4_dequant_ref_cpu`` / ``nf4_dequant_single_cpu``,
SURVEY §8b) and the ``NF4_BACKEND`` switch -- CPU only, no GPU.

Pinned like the oracle: every committed reference fixture bit for bit, and the
C1 / C2 / C3-shape reference digests at full size (tests/golden/manifest.json,
produced by running the reference fallback _aggressive_pytorch_t4,
kernel_optimized.py:208-314).  The product code is what runs here; the oracle
only supplies nothing but the fixture inputs' generator.
"""
import ctypes

import numpy as np
import pytest
import torch
from types import SimpleNamespace

import workloads as W
from _helpers import assert_bits_equal, big_samples, load_case, out_bits, sha, torch_dtype


@pytest.fixture
def cpu_backend(monkeypatch):
    monkeypatch.setenv("NF4_BACKEND", "cpu")
    monkeypatch.setenv("NF4_CPU_THREADS", "4")


def _module(packed, absmax, a2, m, n, dt, a2_f16=None):
    a2_t = torch.from_numpy(a2_f16) if a2_f16 is not None else torch.from_numpy(a2)
    qs = SimpleNamespace(absmax=torch.from_numpy(absmax), state2=SimpleNamespace(absmax=a2_t), dtype=dt)
    return SimpleNamespace(weight=SimpleNamespace(data=torch.from_numpy(packed).view(-1, 1), quant_state=qs),
                           out_features=m, in_features=n)


def test_every_reference_fixture_bit_exact(manifest, cpu_backend):
    from nf4_triton_dequantization import triton_dequantize_nf4

    ran = 0
    for name, e in manifest["cases"].items():
        if "file" not in e:
            continue
        z = load_case(e)
        absmax = z["absmax_f32"] if "absmax_f32" in z else z["a1"]
        mod = _module(z["packed"], absmax, z["a2"], e["m"], e["n"], torch_dtype(e["dtype"]), z.get("a2_f16"))
        out = triton_dequantize_nf4(mod)
        assert out.shape == (e["m"], e["n"]) and out.is_contiguous() and out.device.type == "cpu"
        assert_bits_equal(out_bits(out), z["out_bits"], e["dtype"], name)
        ran += 1
    assert ran >= 18


@pytest.mark.parametrize("name", ["C1_1024x1024_f16", "C2_4096x4096_bf16", "C4_4096x4096_f16", "c64x11008_bf16",
                                  "c1024x4096_f16_neg", "C3_1024x4096_bf16", "C3_14336x4096_bf16",
                                  "C3b_4096x11008_bf16"])
def test_full_size_reference_digests(manifest, cpu_backend, name):
    from nf4_triton_dequantization import triton_dequantize_nf4

    e = manifest["cases"][name]
    m, n = e["m"], e["n"]
    import nf4_oracle as O  # fixture inputs only (the generator + golden overrides)

    p, a1, a2, _ = O.golden_case_inputs(m, n, e["seed"], e["overrides"])
    got = out_bits(triton_dequantize_nf4(_module(p, a1, a2, m, n, torch_dtype(e["dtype"]))))
    idx, bits = big_samples(name)
    assert np.array_equal(got.reshape(-1)[idx], bits)
    assert sha(got) == e["sha256"], name


def test_thread_counts_agree_and_fp32_output():
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    m, n = 77, 64 * 9 + 32  # partial last block, several workers, odd row count
    p, a1, a2 = W.make_inputs(m, n, 9, nb=1001, n2=13, a2_kind="normal")
    outs = []
    for dt, np_t in ((_lib.BF16, np.uint16), (_lib.F16, np.uint16), (_lib.F32, np.uint32)):
        ref = None
        for threads in (1, 3, 8, 0):
            o = np.empty((m, n), np_t)
            rc = L.nf4_dequant_ref_cpu(p.ctypes.data, p.size, a1.ctypes.data, a1.size, a2.ctypes.data, a2.size,
                                       o.ctypes.data, dt, m, n, threads)
            assert rc == 0
            ref = o if ref is None else ref
            assert np.array_equal(o, ref), (dt, threads)
        outs.append(ref)
    # fp32 output is the unrounded product; bf16 is its RNE rounding
    f32 = outs[2].view(np.float32)
    bf = outs[0]
    u = f32.view(np.uint32).astype(np.uint64)
    want = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    assert np.array_equal(bf, want)


def test_single_quant_host_path(cpu_backend):
    from nf4_triton_dequantization import triton_dequantize_nf4

    m, n = 6, 200
    bpr = (n + 63) // 64
    p = W.splitmix64_bytes(3, m * n // 2, stream=1)
    absmax = W.uniform_f32(4, m * (bpr + 2), 0.01, 2.0)
    out = triton_dequantize_nf4(_module(p, absmax, np.zeros(1, np.float32), m, n, torch.float16))
    # direct restatement: scale of (r, b) = absmax[r, b], high nibble first
    lut = torch.tensor([-1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
                        -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
                        0.07958029955625534, 0.16093020141124725, 0.24611230194568634, 0.33791524171829224,
                        0.44070982933044434, 0.5626170039176941, 0.7229568362236023, 1.0], dtype=torch.float32)
    q = torch.from_numpy(p).view(m, n // 2).long()
    nib = torch.stack([q >> 4, q & 15], dim=2).reshape(m, n)
    sc = torch.from_numpy(absmax).view(m, -1)[:, :bpr].repeat_interleave(64, dim=1)[:, :n]
    want = (lut[nib] * sc).to(torch.float16)
    assert torch.equal(out.view(torch.int16), want.view(torch.int16))


def test_fp64_output_is_the_widened_fp32_product(cpu_backend):
    from nf4_triton_dequantization import triton_dequantize_nf4

    m, n = 8, 128
    p, a1, a2 = W.make_inputs(m, n, 5)
    o64 = triton_dequantize_nf4(_module(p, a1, a2, m, n, torch.float64))
    o32 = triton_dequantize_nf4(_module(p, a1, a2, m, n, torch.float32))
    assert o64.dtype == torch.float64 and torch.equal(o64, o32.double())


def test_default_backend_keeps_reference_error(monkeypatch):
    from nf4_triton_dequantization import triton_dequantize_nf4

    monkeypatch.delenv("NF4_BACKEND", raising=False)
    p, a1, a2 = W.make_inputs(2, 64, 1)
    with pytest.raises(RuntimeError, match="ROCm device"):
        triton_dequantize_nf4(_module(p, a1, a2, 2, 64, torch.bfloat16))
    monkeypatch.setenv("NF4_BACKEND", "tpu")
    with pytest.raises(ValueError, match="NF4_BACKEND"):
        triton_dequantize_nf4(_module(p, a1, a2, 2, 64, torch.bfloat16))


def test_host_path_errors_and_many(cpu_backend):
    from nf4_triton_dequantization import triton_dequantize_nf4
    from nf4_triton_dequantization_amd import _lib, dequantize_nf4_many

    p, a1, a2 = W.make_inputs(4, 128, 2)
    # un-viewable packed length -> RuntimeError (the reference's .view raises)
    with pytest.raises(RuntimeError, match="shape"):
        triton_dequantize_nf4(_module(p[:-1], a1, a2, 4, 128, torch.bfloat16))
    with pytest.raises(ZeroDivisionError):
        triton_dequantize_nf4(_module(p, a1[:0], a2, 4, 128, torch.bfloat16))
    L = _lib.lib()
    o = np.empty(8, np.uint16)
    assert L.nf4_dequant_ref_cpu(p.ctypes.data, p.size, a1.ctypes.data, 1, a2.ctypes.data, 1, o.ctypes.data, 7, 4,
                                 128, 1) == _lib.ERR_ARG
    assert L.nf4_dequant_ref_cpu(None, 0, None, 0, None, 0, None, _lib.BF16, 0, 128, 1) == _lib.OK
    mods = [_module(*W.make_inputs(m, n, 40 + m), m, n, torch.bfloat16) for m, n in ((4, 128), (9, 256))]
    outs = dequantize_nf4_many(mods)
    for mod, o in zip(mods, outs):
        assert torch.equal(o, triton_dequantize_nf4(mod))


def test_many_into_caller_outputs(cpu_backend):
    """dequantize_nf4_many(out=...): caller-owned outputs written in place and returned;
    a wrong shape / dtype / layout raises before anything runs."""
    from nf4_triton_dequantization import triton_dequantize_nf4
    from nf4_triton_dequantization_amd import dequantize_nf4_many

    mods = [_module(*W.make_inputs(m, n, 60 + m), m, n, torch.bfloat16) for m, n in ((4, 128), (9, 256), (3, 64))]
    bufs = [torch.full((4, 128), 7.0, dtype=torch.bfloat16), None, torch.empty((3, 64), dtype=torch.bfloat16)]
    outs = dequantize_nf4_many(mods, out=bufs)
    assert outs[0] is bufs[0] and outs[2] is bufs[2]
    for mod, o in zip(mods, outs):
        assert torch.equal(o, triton_dequantize_nf4(mod))
    for bad in (torch.empty((4, 127), dtype=torch.bfloat16), torch.empty((4, 128), dtype=torch.float16),
                torch.empty((128, 4), dtype=torch.bfloat16).t()):
        with pytest.raises(RuntimeError, match="out\\[0\\]"):
            dequantize_nf4_many(mods[:1], out=[bad])
    with pytest.raises(ValueError):
        dequantize_nf4_many(mods, out=bufs[:2])
