"""Maximum sizes (``-m gpu``): matrices past one buffer descriptor's reach.

A flat piece holds < 2^29 packed bytes (its output must stay under 4 GiB of
buffer range); bigger matrices -- e.g. a 70B model's 128256 x 8192 lm_head --
go as row-aligned pieces of one launch, each carrying its first scale block.
These tests cross the piece boundary with the reference's wrap semantics
(absmax counts that are not multiples of anything), in every scale mode, and
compare all ~1.07e9 outputs with the C oracle bit for bit.
"""
import numpy as np
import pytest
import torch

import nf4_oracle as O
from _helpers import assert_bits_equal, make_module, out_bits

pytestmark = pytest.mark.gpu

M_BIG, N_BIG = 262144 + 100, 4096  # 537,075,712 packed bytes: pieces of 262,143 and 101 rows


@pytest.fixture(scope="module")
def big_inputs():
    return O.make_inputs(M_BIG, N_BIG, 5, nb=1000003, n2=4099, a2_kind="normal")


def _equal_on_device(out: torch.Tensor, want: np.ndarray, what: str):
    w = torch.from_numpy(want.view(np.int16)).to(out.device).view(out.shape)
    diff = out.view(torch.int16) != w
    if bool(diff.any()):
        bad = diff.nonzero()[:8].tolist()
        raise AssertionError(f"{what}: {int(diff.sum())} outputs differ, first at {bad}")


def test_ref_semantics_across_pieces(coracle, gpu, big_inputs):
    import nf4_triton_dequantization as N

    p, a1, a2 = big_inputs
    assert p.nbytes >= 1 << 29
    coracle.set_threads(16)
    want = coracle.dequant_ref(p, a1, a2, M_BIG, N_BIG, O.BF16)
    out = N.triton_dequantize_nf4(make_module(p, a1, a2, M_BIG, N_BIG, "bf16", gpu))
    torch.cuda.synchronize()
    _equal_on_device(out, want, "ref bf16")
    del out


def test_batched_with_a_big_member(coracle, gpu, big_inputs):
    from nf4_triton_dequantization_amd import dequantize_nf4_many

    p, a1, a2 = big_inputs
    coracle.set_threads(16)
    small = [O.golden_case_inputs(m, n, 900 + m, {"stride": n // 2}) for (m, n) in ((64, 4096), (33, 11008))]
    mods = [make_module(p, a1, a2, M_BIG, N_BIG, "f16", gpu)]
    mods += [make_module(sp, sa1, sa2, m, n, "f16", gpu) for (sp, sa1, sa2, _), (m, n) in
             zip(small, ((64, 4096), (33, 11008)))]
    outs = dequantize_nf4_many(mods)
    torch.cuda.synchronize()
    _equal_on_device(outs[0], coracle.dequant_ref(p, a1, a2, M_BIG, N_BIG, O.F16), "batched big member")
    for (sp, sa1, sa2, _), (m, n), o in zip(small, ((64, 4096), (33, 11008)), outs[1:]):
        assert_bits_equal(out_bits(o), coracle.dequant_ref(sp, sa1, sa2, m, n, O.F16), "f16", f"{m}x{n}")


def test_single_quant_across_pieces(coracle, gpu, big_inputs):
    import nf4_triton_dequantization as N

    p, _, _ = big_inputs
    bpr = N_BIG // 64
    absmax = O.uniform_f32(77, M_BIG * (bpr + 3), 0.01, 2.0)  # rows of bpr + 3 (the reference slices :bpr)
    coracle.set_threads(16)
    want = coracle.dequant_single(p, absmax, M_BIG, N_BIG, O.F16)
    mod = make_module(p, absmax, np.zeros(1, np.float32), M_BIG, N_BIG, "f16", gpu)
    out = N.triton_dequantize_nf4(mod)
    torch.cuda.synchronize()
    _equal_on_device(out, want, "single f16")


def test_bnb_stream_across_pieces(coracle, gpu, big_inputs):
    from nf4_triton_dequantization_amd import _lib

    p, _, _ = big_inputs
    numel = 2 * p.size  # 1,074,151,424 elements: 2^28-byte pieces
    nblk = (numel + 63) // 64
    a1 = O.splitmix64_bytes(31, nblk, stream=2)
    code2 = np.sort(O.normal_f32(32, 256)).astype(np.float32)
    a2 = O.uniform_f32(33, (nblk + 255) // 256, 0.01, 0.1)
    coracle.set_threads(16)
    want = coracle.dequant_bnb(p, a1, code2, a2, 0.03125, numel, O.BF16)
    t = [torch.from_numpy(x).to(gpu) for x in (p, a1, code2, a2)]
    out = torch.empty(numel, dtype=torch.bfloat16, device=gpu)
    rc = _lib.lib().nf4_dequant_bnb(t[0].data_ptr(), t[1].data_ptr(), t[1].numel(), t[2].data_ptr(),
                                    t[3].data_ptr(), t[3].numel(), 0.03125, out.data_ptr(), _lib.BF16, numel, 64,
                                    256, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    _equal_on_device(out, want, "bnb bf16")
