"""Concurrent streams and hipGraph capture through the product API (``-m gpu``).

* The fused GEMM keeps split-K ticket counters in a per-(device, stream)
  workspace; calls on several streams at once must neither share counters nor
  lose determinism: each stream's results equal a serial run bit for bit
  (the library's split-K sum is in slice order, so reproducible by design).
* Decode passes are replayed as hipGraphs (tools/bench_gemm.py): the drop-in
  dequant, the batched dequant and the fused GEMM captured into one graph and
  replayed must give the eager results bit for bit.
"""
import numpy as np
import pytest
import torch

import nf4_oracle as O
from _helpers import make_module

pytestmark = pytest.mark.gpu

# (M, N, K): the library's split-K choices -- persistent with K slices (12 rows),
# register-resident with two K slices (32 rows), streaming down projection (1 row)
SHAPES = [(12, 4096, 4096), (32, 2048, 4096), (1, 4096, 14336)]


def _mods(gpu):
    mods, xs = [], []
    for i, (M, N, K) in enumerate(SHAPES):
        packed, a1, a2 = O.make_inputs(N, K, seed=500 + i, a2_kind="normal")
        mods.append(make_module(packed, a1, a2, N, K, "bf16", gpu))
        xs.append(torch.from_numpy(O.normal_f32(600 + i, M * K, stream=9).reshape(M, K)).to(torch.bfloat16).to(gpu))
    return mods, xs


def test_fused_gemm_on_concurrent_streams_is_bitwise_serial(gpu):
    from nf4_triton_dequantization_amd import nf4_linear

    mods, xs = _mods(gpu)
    serial = [nf4_linear(x, m) for x, m in zip(xs, mods)]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(gpu) for _ in SHAPES]
    main = torch.cuda.current_stream(gpu)
    outs = [[] for _ in SHAPES]
    for _ in range(12):
        for i, s in enumerate(streams):
            s.wait_stream(main)
            with torch.cuda.stream(s):
                outs[i].append(nf4_linear(xs[i], mods[i]))
    for s in streams:
        main.wait_stream(s)
    torch.cuda.synchronize()
    for i, ys in enumerate(outs):
        for y in ys:
            assert torch.equal(y.view(torch.int16), serial[i].view(torch.int16)), f"stream {i}: not bitwise serial"


def test_graph_capture_replays_bitwise(gpu):
    from nf4_triton_dequantization import triton_dequantize_nf4
    from nf4_triton_dequantization_amd import dequantize_nf4_many, nf4_linear, nf4_linear_grouped

    mods, xs = _mods(gpu)
    small = []
    for i, (m, n) in enumerate([(1024, 4096), (96, 320), (4096, 4096)]):
        packed, a1, a2 = O.make_inputs(m, n, seed=700 + i)
        small.append(make_module(packed, a1, a2, m, n, "bf16", gpu))
    x0 = xs[1][:5].contiguous()
    grouped_mods = [mods[1], small[0]] if small[0].in_features == mods[1].in_features else [mods[1]]

    def body():
        a = triton_dequantize_nf4(small[2])
        b = dequantize_nf4_many(small)
        c = [nf4_linear(x, m) for x, m in zip(xs, mods)]
        d = nf4_linear_grouped(x0, grouped_mods)
        return [a, *b, *c, *d]

    s = torch.cuda.Stream(gpu)
    s.wait_stream(torch.cuda.current_stream(gpu))
    with torch.cuda.stream(s):
        eager = body()  # also creates this stream's GEMM workspace outside the capture
        eager = [t.clone() for t in eager]
    torch.cuda.current_stream(gpu).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        captured = body()
    for _ in range(3):
        for t in captured:
            t.zero_()
        g.replay()
        torch.cuda.synchronize()
        for k, (want, got) in enumerate(zip(eager, captured)):
            assert torch.equal(got.view(torch.int16), want.view(torch.int16)), f"output {k} differs after replay"
    assert np.isfinite(float(captured[0].float().abs().max()))
