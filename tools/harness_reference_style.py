"""The reference harness's timed loop, replayed on MI355X with this path.

Restates the measurement of the reference's benchmark.py (:86-138): for each of
its three MLP configs (hd, m, dtype) = (2048, 8192, fp16), (1024, 4096, bf16),
(4096, 14336, bf16), three Linear4bit weights (gate, up: m x hd; down: hd x m)
are dequantized per iteration on three fresh streams (:68-84, ``.t()`` of each
result), ``iterations`` times between two events; the total seconds is the
number the reference compares against unsloth.  unsloth/peft/bitsandbytes are
absent here, so only this path's time is reported, together with the device
time the same dequantizations need (hipGraph replay) -- the gap between the two
is host launch overhead (Python + ctypes + allocation per call).  Unlike the
reference loop, the end event waits for all three streams.

Also reports the per-call host cost of ``triton_dequantize_nf4`` alone.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from nf4_triton_dequantization import triton_dequantize_nf4  # noqa: E402
from nf4_triton_dequantization_amd import Linear4bit, dequantize_nf4_many  # noqa: E402

OPTIONS = [(2, 3333, 2048, 8192, 3407, torch.float16),
           (5, 777, 1024, 4096, 3409, torch.bfloat16),
           (3, 2048, 4096, 14336, 3408, torch.bfloat16)]


class MLP(torch.nn.Module):
    def __init__(self, hd, m, dtype):
        super().__init__()
        self.gate_proj = Linear4bit(hd, m, compute_dtype=dtype).to("cuda")
        self.up_proj = Linear4bit(hd, m, compute_dtype=dtype).to("cuda")
        self.down_proj = Linear4bit(m, hd, compute_dtype=dtype).to("cuda")


def mlp_dequantize(mlp, fx, sync=True):
    s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):
        a = fx(mlp.up_proj).t()
    with torch.cuda.stream(s2):
        b = fx(mlp.gate_proj).t()
    with torch.cuda.stream(s3):
        c = fx(mlp.down_proj).t()
    if sync:
        torch.cuda.synchronize()
    else:
        # the timing event is recorded on the current stream: make it wait for the
        # three side streams, or it can fire before their work is done (the
        # reference's benchmark.py:116-126 has that flaw; not copied)
        cur = torch.cuda.current_stream()
        for s in (s1, s2, s3):
            cur.wait_stream(s)
    return a, b, c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iterations", type=int, default=1000)
    args = ap.parse_args()
    total = 0.0
    for bsz, qlen, hd, m, seed, dt in OPTIONS:
        torch.manual_seed(seed)
        mlp = MLP(hd, m, dt)
        for _ in range(2):
            mlp_dequantize(mlp, triton_dequantize_nf4)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iterations):
            mlp_dequantize(mlp, triton_dequantize_nf4, sync=False)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3
        total += t
        # the same loop's pieces: host time to issue it, the three
        # torch.cuda.Stream() creations alone, and the three drop-in calls alone on the
        # current stream (no new streams), each per iteration
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        for _ in range(args.iterations):
            mlp_dequantize(mlp, triton_dequantize_nf4, sync=False)
        host_loop_us = (time.perf_counter() - h0) * 1e6 / args.iterations
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        for _ in range(args.iterations):
            _s = (torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream())
        streams_us = (time.perf_counter() - h0) * 1e6 / args.iterations
        del _s
        # the harness's own plumbing: the same loop with a dequant that returns a ready
        # tensor (3 streams, 3 stream contexts, .t(), 3 wait_stream), no kernel
        ready = torch.empty((2, 2), device="cuda")
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        for _ in range(args.iterations):
            mlp_dequantize(mlp, lambda md: ready, sync=False)
        plumbing_us = (time.perf_counter() - h0) * 1e6 / args.iterations
        torch.cuda.synchronize()
        mods3 = [mlp.up_proj, mlp.gate_proj, mlp.down_proj]
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        for _ in range(args.iterations):
            for md in mods3:
                triton_dequantize_nf4(md).t()
        calls_us = (time.perf_counter() - h0) * 1e6 / args.iterations
        torch.cuda.synchronize()
        # device time of the three single launches (one stream, graph replay)
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            outs1 = [triton_dequantize_nf4(md) for md in mods3]
        g1.replay()
        torch.cuda.synchronize()
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0.record()
        for _ in range(50):
            g1.replay()
        r1.record()
        torch.cuda.synchronize()
        dev1_us = r0.elapsed_time(r1) * 1e3 / 50
        del outs1, g1
        # device-only time of the same three dequantizations (graph replay, batched launch)
        mods = [mlp.up_proj, mlp.gate_proj, mlp.down_proj]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            outs = dequantize_nf4_many(mods)
        g.replay()
        torch.cuda.synchronize()
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0.record()
        for _ in range(50):
            g.replay()
        r1.record()
        torch.cuda.synchronize()
        dev_us = r0.elapsed_time(r1) * 1e3 / 50
        elems = 3 * hd * m
        print(json.dumps({"config": f"hd={hd} m={m} {str(dt).replace('torch.', '')}",
                          "iterations": args.iterations, "seconds": t, "us_per_iteration": t * 1e6 / args.iterations,
                          "device_us_per_iteration_batched_graph": dev_us,
                          "device_us_per_iteration_three_launches_graph": dev1_us,
                          "host_us_per_iteration_issue": host_loop_us,
                          "host_us_three_stream_creations": streams_us,
                          "host_us_three_dropin_calls_current_stream": calls_us,
                          "host_us_harness_plumbing_no_kernel": plumbing_us,
                          "elements_per_iteration": elems}), flush=True)
        del outs, g
    # host cost of one API call (device work hidden behind a long queue)
    lin = Linear4bit(4096, 4096, compute_dtype=torch.bfloat16).to("cuda")
    for _ in range(20):
        triton_dequantize_nf4(lin)
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)
    n = 1000  # stays well inside the hardware queue behind the spin
    t0 = time.perf_counter()
    for _ in range(n):
        triton_dequantize_nf4(lin)
    host_us = (time.perf_counter() - t0) * 1e6 / n
    torch.cuda.synchronize()
    # the same call on a duck-typed module holding plain tensors (no nn.Parameter
    # `.data` re-wrap per call) -- what is left is this path's own cost
    from types import SimpleNamespace

    w = lin.weight
    duck = SimpleNamespace(weight=SimpleNamespace(data=w.data, quant_state=w.quant_state),
                           out_features=lin.out_features, in_features=lin.in_features)
    for _ in range(20):
        triton_dequantize_nf4(duck)
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)
    t0 = time.perf_counter()
    for _ in range(n):
        triton_dequantize_nf4(duck)
    duck_us = (time.perf_counter() - t0) * 1e6 / n
    torch.cuda.synchronize()
    # torch's own floor for comparison: one allocation of the output per call
    torch.cuda._sleep(200_000_000)
    t0 = time.perf_counter()
    for _ in range(n):
        torch.empty((4096, 4096), dtype=torch.bfloat16, device="cuda")
    empty_us = (time.perf_counter() - t0) * 1e6 / n
    torch.cuda.synchronize()
    # and one minimal torch kernel launch (an in-place add on 1 element): the host cost
    # of any single kernel launch from Python on this stack
    tiny = torch.zeros(1, device="cuda")
    torch.cuda._sleep(200_000_000)
    t0 = time.perf_counter()
    for _ in range(n):
        tiny.add_(1.0)
    launch_us = (time.perf_counter() - t0) * 1e6 / n
    torch.cuda.synchronize()
    # the pieces: the tensor-level entry alone (no Python attribute reads), and the
    # bare C-ABI launch into a preallocated output through ctypes
    from nf4_triton_dequantization_amd import _lib
    from nf4_triton_dequantization_amd import kernel as _K

    _EXT = _K._ext()

    qs = w.quant_state
    q, a1, a2 = w.data, qs.absmax, qs.state2.absmax
    ext_us = None
    if _EXT is not None:
        torch.cuda._sleep(200_000_000)
        t0 = time.perf_counter()
        for _ in range(n):
            _EXT.dequant_ref(q, a1, a2, 4096, 4096, _lib.BF16)
        ext_us = (time.perf_counter() - t0) * 1e6 / n
        torch.cuda.synchronize()
    out = torch.empty((4096, 4096), dtype=torch.bfloat16, device="cuda")
    fn = _lib.lib().nf4_dequant_ref
    args = (q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(), out.data_ptr(), _lib.BF16,
            4096, 4096, torch.cuda.current_stream().cuda_stream)
    torch.cuda._sleep(200_000_000)
    t0 = time.perf_counter()
    for _ in range(n):
        fn(*args)
    cabi_us = (time.perf_counter() - t0) * 1e6 / n
    torch.cuda.synchronize()
    print(json.dumps({"reference_style_total_seconds": total, "api_host_us_per_call": host_us,
                      "api_host_us_per_call_plain_tensors": duck_us, "ext_entry_us": ext_us,
                      "c_abi_launch_us_ctypes": cabi_us, "torch_empty_us": empty_us,
                      "torch_min_kernel_launch_us": launch_us, "calls_per_figure": n}), flush=True)


if __name__ == "__main__":
    main()
