"""The reference consumer at its own shapes: ``X @ triton_dequantize_nf4(W).t()``.

    python tools/bench_prefill.py [--reps 20] > profiles/r02/prefill_mlp.jsonl

The reference harness (benchmark.py:61-66, :86-92) multiplies activations of
(bsz, qlen, hd) = (2, 3333, 2048) fp16, (5, 777, 1024) bf16 and (3, 2048, 4096)
bf16 -- M = 6666, 3885, 6144 rows -- by the dequantized gate / up / down weights
of an MLP (m = 8192, 4096, 14336).  At these M the product is a large GEMM
(hipBLASLt, MFMA-bound) and the dequantization is a small add-on, so this path
keeps the composite: one dequant launch per weight + torch.matmul.  This tool
measures, per config, the MLP forward (up, gate, silu(gate) * up, down) with

* ``bf16``:      the weights already dequantized (no quantization at all);
* ``composite``: triton_dequantize_nf4 per weight inside the forward (nf4_linear's
  large-M path), as the reference's mlp_forward does;
* ``dequant``:   the three dequantizations alone (one batched launch);

all captured in hipGraphs (median of --reps replays), and checks that the
composite's output equals the bf16 forward bit for bit (same weights, same GEMMs).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from nf4_triton_dequantization import triton_dequantize_nf4  # noqa: E402
from nf4_triton_dequantization_amd import Linear4bit, dequantize_nf4_many  # noqa: E402

OPTIONS = [(2, 3333, 2048, 8192, 3407, torch.float16),
           (5, 777, 1024, 4096, 3409, torch.bfloat16),
           (3, 2048, 4096, 14336, 3408, torch.bfloat16)]


def graph_time(fn, reps):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2], out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    act = torch.nn.functional.silu
    for bsz, qlen, hd, m, seed, dt in OPTIONS:
        torch.manual_seed(seed)
        up = Linear4bit(hd, m, compute_dtype=dt, device=dev)
        gate = Linear4bit(hd, m, compute_dtype=dt, device=dev)
        down = Linear4bit(m, hd, compute_dtype=dt, device=dev)
        x = torch.randn((bsz * qlen, hd), device=dev, dtype=dt)
        wu, wg, wd = (triton_dequantize_nf4(lin) for lin in (up, gate, down))

        def fwd_bf16():
            return (act(x @ wg.t()) * (x @ wu.t())) @ wd.t()

        def fwd_composite():
            u = x @ triton_dequantize_nf4(up).t()
            g = x @ triton_dequantize_nf4(gate).t()
            return (act(g) * u) @ triton_dequantize_nf4(down).t()

        def deq_only():
            return dequantize_nf4_many([up, gate, down])

        t_bf16, y_ref = graph_time(fwd_bf16, args.reps)
        t_comp, y_comp = graph_time(fwd_composite, args.reps)
        t_deq, _ = graph_time(deq_only, args.reps)
        same = bool(torch.equal(y_ref, y_comp))
        M = bsz * qlen
        flops = 2 * M * hd * m * 3
        print(json.dumps({"config": f"bsz={bsz} qlen={qlen} hd={hd} m={m} {str(dt).replace('torch.', '')}", "M": M,
                          "bf16_weights_us": round(t_bf16, 1), "composite_us": round(t_comp, 1),
                          "dequant_only_us": round(t_deq, 1), "composite_over_bf16": round(t_comp / t_bf16, 4),
                          "dequant_share_of_composite": round(t_deq / t_comp, 4),
                          "gemm_tflops_bf16_weights": round(flops / t_bf16 / 1e6, 1),
                          "composite_equals_bf16_forward": same}), flush=True)
        assert same, "composite forward differs from the forward on the same dequantized weights"
        del up, gate, down, wu, wg, wd
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
