"""Does a decode GEMM launch gain from its weight being in the Infinity Cache (MALL)?

    python tools/mall_prefetch_probe.py [--ms 1,32] [--shape 14336,4096]

Per M, three hipGraph-replayed sequences of fused GEMM launches (library default
decomposition), microseconds per launch:
  * stream:   each launch on a different weight (> MALL in total: HBM-streamed)
  * resident: every launch on the same weight (its 29 MB stay in MALL / L2)
  * prefetch: distinct weights, and while launch i runs, a side stream reads
              weight i + 1 (a torch reduction), which launch i + 1 waits for
A large stream/resident gap with prefetch near resident says the next weight's
read can be overlapped with the current launch (tools only: a probe, not a product
path).
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


def graph_us(body, n_launch, reps=7):
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
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
    return ts[len(ts) // 2] * 1e3 / n_launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,32")
    ap.add_argument("--shape", default="14336,4096")
    ap.add_argument("--copies", type=int, default=27)
    args = ap.parse_args()
    n, k = (int(v) for v in args.shape.split(","))
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    nb = n * k // 64
    ws = [(torch.randint(0, 256, (n * k // 2,), dtype=torch.uint8, device=dev, generator=gen),
           torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=gen),
           torch.rand((nb + 255) // 256, device=dev, generator=gen) * 0.01 + 1e-3) for _ in range(args.copies)]
    C = len(ws)
    side = torch.cuda.Stream(dev)
    acc = torch.zeros(C, dtype=torch.int64, device=dev)
    for M in [int(v) for v in args.ms.split(",")]:
        x = torch.randn((M, k), device=dev).to(torch.bfloat16)
        y = torch.empty((M, n), dtype=torch.bfloat16, device=dev)
        wsb = L.nf4_gemm_workspace_bytes(M, n, k)
        wk = torch.zeros(max(wsb, 1 << 16), dtype=torch.uint8, device=dev)

        def gemm(i):
            q, a1, a2 = ws[i]
            rc = L.nf4_gemm_ref(x.data_ptr(), M, q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(),
                                a2.numel(), y.data_ptr(), _lib.BF16, n, k, wk.data_ptr(), wsb,
                                torch.cuda.current_stream().cuda_stream)
            assert rc == 0, rc

        def stream_body():
            for i in range(C):
                gemm(i)

        def resident_body():
            for _ in range(C):
                gemm(0)

        def prefetch_body():
            main_st = torch.cuda.current_stream()
            ready = [torch.cuda.Event() for _ in range(C)]
            started = [torch.cuda.Event() for _ in range(C)]
            with torch.cuda.stream(side):
                side.wait_stream(main_st)
                torch.sum(ws[0][0].view(torch.int32), dim=0, dtype=torch.int64, out=acc[0])
                ready[0].record(side)
            for i in range(C):
                main_st.wait_event(ready[i])
                started[i].record(main_st)
                if i + 1 < C:
                    with torch.cuda.stream(side):
                        side.wait_event(started[i])
                        torch.sum(ws[i + 1][0].view(torch.int32), dim=0, dtype=torch.int64, out=acc[i + 1])
                        ready[i + 1].record(side)
                gemm(i)
            main_st.wait_stream(side)

        def prefetch_only():
            for i in range(C):
                torch.sum(ws[i][0].view(torch.int32), dim=0, dtype=torch.int64, out=acc[i])

        out = {"N": n, "K": k, "M": M, "copies": C,
               "stream_us": round(graph_us(stream_body, C), 2),
               "resident_us": round(graph_us(resident_body, C), 2),
               "prefetch_us": round(graph_us(prefetch_body, C), 2),
               "read_only_us": round(graph_us(prefetch_only, C), 2)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
