"""BASELINE configs at full size (``-m gpu``): the whole C3 pass.

C3 = every linear weight of Llama-3-8B (32 layers x 7 = 224 matrices, 6.98e9
elements; BASELINE configs[2]) and C3b = the 4096/11008 set BASELINE names
(Llama-2-7B shapes), each dequantized in ONE call of ``dequantize_nf4_many`` --
the batched launches bench/tools time (<= NF4DQ_BATCH_MAX matrices per launch,
so 10 launches for 224 weights) -- with distinct inputs per matrix, and every
output compared bit for bit with the C oracle (the oracle itself is pinned to
the reference fallback at each of these shapes: tests/golden/manifest.json
C3_* / C3b_* digests, tests/test_oracle_golden.py).  Comparison happens on the
device, one matrix at a time, so host memory stays at one oracle output.

C2 / C4 / C5 single matrices are pinned to the reference's own digests in
tests/test_gpu_parity.py::test_full_size_matches_reference_digest.
"""
import numpy as np
import pytest
import torch

import nf4_oracle as O
import workloads as W
from _helpers import make_module

pytestmark = pytest.mark.gpu


def _equal_on_device(out: torch.Tensor, want: np.ndarray, what: str):
    w = torch.from_numpy(want.view(np.int16)).to(out.device).view(out.shape)
    diff = out.view(torch.int16) != w
    if bool(diff.any()):
        bad = diff.nonzero()[:8].tolist()
        raise AssertionError(f"{what}: {int(diff.sum())} outputs differ, first at {bad}")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("variant,seed0", [("llama3", 50000), ("llama2", 60000)])
def test_c3_full_pass_batched_vs_oracle(coracle, gpu, variant, seed0):
    from nf4_triton_dequantization_amd import _lib, dequantize_nf4_many

    shapes = W.c3_shapes(variant)
    assert len(shapes) == 224
    inputs = [W.make_inputs(m, n, seed0 + i) for i, (m, n) in enumerate(shapes)]
    mods = [make_module(p, a1, a2, m, n, "bf16", gpu) for (p, a1, a2), (m, n) in zip(inputs, shapes)]
    outs = dequantize_nf4_many(mods)
    torch.cuda.synchronize()
    assert len(outs) == 224 and -(-224 // _lib.BATCH_MAX) == 10
    coracle.set_threads(16)
    total = 0
    for i, ((p, a1, a2), (m, n), o) in enumerate(zip(inputs, shapes, outs)):
        assert o.shape == (m, n) and o.dtype == torch.bfloat16 and o.is_contiguous()
        _equal_on_device(o, coracle.dequant_ref(p, a1, a2, m, n, O.BF16), f"{variant} weight {i} {m}x{n}")
        total += m * n
    assert total == {"llama3": 6_979_321_856, "llama2": 6_476_005_376}[variant]
