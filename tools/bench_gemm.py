"""Fused NF4 dequant-GEMM (decode shapes) vs the unfused alternatives, one MI355X.

    python tools/bench_gemm.py [--layers 32] [--ms 1,4,8,16,32]

Workload: every linear of Llama-3-8B (32 layers x {q,o 4096x4096; k,v
1024x4096; gate,up 14336x4096; down 4096x14336}), y = x @ W^T for a decode
batch of M rows.  All 224 weights are distinct buffers (3.5 GB packed), so
each pass streams them from HBM.  Per M, hipGraph replay of one full pass:

  fused      nf4_gemm_ref per weight (4-bit weight read once, dequant in registers)
  grouped    nf4_gemm_ref_grouped: q/k/v in one launch, gate/up in one (they share x), o and down alone
  composite  nf4_dequant_ref + torch.matmul per weight (the reference harness's pattern)
  bf16       torch.matmul on pre-dequantized bf16 weights (no quantization; 4x the weight bytes)

Roofline of the fused kernel: HBM bytes = N*K/2 packed + N*K/64 absmax + nested
absmax + x + y per weight, vs 8 TB/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from nf4_triton_dequantization_amd import _lib  # noqa: E402

SHAPES = [(4096, 4096), (1024, 4096), (1024, 4096), (4096, 4096), (14336, 4096), (14336, 4096), (4096, 14336)]
PEAK = 8e12


def graph_ms(fn, reps=5):
    fn()  # eager first: library handles/workspaces (hipBLASLt) cannot be created under capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--ms", default="1,4,8,16,32")
    ap.add_argument("--no-bf16", action="store_true")
    ap.add_argument("--no-composite", action="store_true")
    ap.add_argument("--lib", default="prod", help="prod, or a tools/_build/libnf4dq_<name>.so variant (A/B runs)")
    args = ap.parse_args()
    if args.lib != "prod":
        _lib.LIB_PATH = os.path.join(REPO, "tools", "_build", f"libnf4dq_{args.lib}.so")
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    ws = []
    for _ in range(args.layers):
        for (n, k) in SHAPES:
            nb = n * k // 64
            ws.append((n, k, torch.randint(0, 256, (n * k // 2,), dtype=torch.uint8, device=dev, generator=gen),
                       torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=gen),
                       torch.rand((nb + 255) // 256, device=dev, generator=gen) * 0.01 + 1e-3))
    wbf = None
    if not args.no_bf16:
        wbf = []
        for (n, k, q, a1, a2) in ws:
            w = torch.empty((n, k), dtype=torch.bfloat16, device=dev)
            assert L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                     w.data_ptr(), _lib.BF16, n, k, torch.cuda.current_stream().cuda_stream) == 0
            wbf.append(w)
    tmp = {(n, k): torch.empty((n, k), dtype=torch.bfloat16, device=dev) for (n, k) in set(SHAPES)}
    packed_bytes = sum(q.numel() + a1.numel() + 4 * a2.numel() for (_, _, q, a1, a2) in ws)
    for M in [int(v) for v in args.ms.split(",")]:
        xs = {k: torch.randn((M, k), device=dev).to(torch.bfloat16) for k in {k for _, k in SHAPES}}
        ys = [torch.empty((M, n), dtype=torch.bfloat16, device=dev) for (n, _, _, _, _) in ws]
        wsz = max(L.nf4_gemm_workspace_bytes(M, n, k) for (n, k) in SHAPES)
        work = torch.zeros(max(wsz, 1), dtype=torch.uint8, device=dev)  # zero before first use (counters)

        def fused():
            sp = torch.cuda.current_stream().cuda_stream
            for i, (n, k, q, a1, a2) in enumerate(ws):
                x = xs[k]
                rc = L.nf4_gemm_ref(x.data_ptr(), M, q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(),
                                    a2.data_ptr(), a2.numel(), ys[i].data_ptr(), _lib.BF16, n, k, work.data_ptr(),
                                    wsz, sp)
                assert rc == 0, rc

        # q,k,v (0,1,2) and gate,up (4,5) share their input: one launch each
        groups = []
        for layer in range(args.layers):
            b = layer * len(SHAPES)
            for idx in ((0, 1, 2), (3,), (4, 5), (6,)):
                mats = (_lib.GemmMat * len(idx))()
                for j, i in enumerate(idx):
                    n, k, q, a1, a2 = ws[b + i]
                    mats[j] = _lib.GemmMat(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(),
                                           a2.numel(), ys[b + i].data_ptr(), n)
                groups.append((ws[b + idx[0]][1], mats, len(idx)))
        gwsz = max(L.nf4_gemm_grouped_workspace_bytes(M, k, mats, c, None) for (k, mats, c) in groups)
        gwork = torch.zeros(max(gwsz, 1), dtype=torch.uint8, device=dev)

        def grouped():
            sp = torch.cuda.current_stream().cuda_stream
            for (k, mats, c) in groups:
                rc = L.nf4_gemm_ref_grouped(xs[k].data_ptr(), M, k, mats, c, _lib.BF16, gwork.data_ptr(), gwsz,
                                            None, sp)
                assert rc == 0, rc

        def composite():
            sp = torch.cuda.current_stream().cuda_stream
            for i, (n, k, q, a1, a2) in enumerate(ws):
                w = tmp[(n, k)]
                assert L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(),
                                         a2.numel(), w.data_ptr(), _lib.BF16, n, k, sp) == 0
                torch.matmul(xs[k], w.t(), out=ys[i])

        def bf16():
            for i, (n, k, *_r) in enumerate(ws):
                torch.matmul(xs[k], wbf[i].t(), out=ys[i])

        io_bytes = sum(M * k * 2 + M * n * 2 for (n, k, *_r) in ws)
        res = {"M": M, "weights": len(ws)}
        t = graph_ms(fused)
        res.update({"fused_ms": t, "fused_TBps": (packed_bytes + io_bytes) / (t * 1e-3) / 1e12,
                    "fused_frac": (packed_bytes + io_bytes) / (t * 1e-3) / PEAK})
        tg = graph_ms(grouped)
        res.update({"grouped_ms": tg, "grouped_TBps": (packed_bytes + io_bytes) / (tg * 1e-3) / 1e12,
                    "grouped_launches": len(groups)})
        res["lib"] = args.lib
        if not args.no_composite:
            res["composite_ms"] = graph_ms(composite)
            res["speedup_vs_composite"] = res["composite_ms"] / t
        if wbf is not None:
            res["bf16_weights_ms"] = graph_ms(bf16)
        if wbf is not None:
            res["speedup_vs_bf16_weights"] = res["bf16_weights_ms"] / t
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
