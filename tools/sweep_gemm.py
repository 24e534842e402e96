"""Sweep the fused GEMM decomposition (waves per workgroup, chunks in flight, K split).

    python tools/sweep_gemm.py [--ms 1,16,32] [--copies 48]

Per (N, K) of Llama-3-8B and per M, every valid nf4_gemm_cfg is timed on
`copies` distinct weights (> MALL, so each launch streams its weight from HBM)
under hipGraph replay; prints one JSON line per (shape, M) with all configs
sorted by time and the library default's rank.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from nf4_triton_dequantization_amd import _lib  # noqa: E402

SHAPES = [(4096, 4096), (1024, 4096), (14336, 4096), (4096, 14336), (6144, 4096), (28672, 4096)]
# (6144, 4096) / (28672, 4096): the column totals of the grouped q/k/v and gate/up
# launches (default_gemm_cfg is keyed by the launch's total N)


def graph_us(fn, n_launch, reps=5):
    fn()
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
    return ts[len(ts) // 2] * 1e3 / n_launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,16,32")
    ap.add_argument("--budget-mb", type=int, default=768, help="packed weight bytes per shape")
    ap.add_argument("--shapes", default="", help="N,K;N,K;... (default: the Llama-3-8B list)")
    ap.add_argument("--kernels", default="1,2,3,4,5",
                    help="kernel ids to sweep (1 K128, 2 stream, 3 persist, 4 shared-activation, "
                         "5 register-resident)")
    args = ap.parse_args()
    shapes = [tuple(int(v) for v in s.split(",")) for s in args.shapes.split(";")] if args.shapes else SHAPES
    kern = {int(v) for v in args.kernels.split(",")}
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    for (n, k) in shapes:
        copies = max(8, args.budget_mb * (1 << 20) // (n * k // 2))
        nb = n * k // 64
        ws = [(torch.randint(0, 256, (n * k // 2,), dtype=torch.uint8, device=dev, generator=gen),
               torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=gen),
               torch.rand((nb + 255) // 256, device=dev, generator=gen) * 0.01 + 1e-3) for _ in range(copies)]
        wbytes = n * k // 2 + nb + 4 * ((nb + 255) // 256)
        for M in [int(v) for v in args.ms.split(",")]:
            x = torch.randn((M, k), device=dev).to(torch.bfloat16)
            y = torch.empty((M, n), dtype=torch.bfloat16, device=dev)
            ref = None
            res = []
            cfgs = []
            for waves in (4, 8, 16):
                for depth in (2, 4):
                    for strips in (1, 2, 4):
                        for ks in (1, 2, 4):
                            cfgs.append(_lib.GemmCfg(_lib.GEMM_PERSIST, waves, depth, ks, strips))
            for waves in (4, 8, 16):
                for depth in (2, 4, 8):
                    for strips in (1, 2, 4):
                        for ks in (1, 2, 4, 8):
                            cfgs.append(_lib.GemmCfg(_lib.GEMM_STREAM, waves, depth, ks, strips))
            for waves in (4, 8):
                for depth in (1, 2):
                    for strips in (1, 2, 4):  # K128: strips per wave
                        for ks in (1, 2, 4, 8):
                            cfgs.append(_lib.GemmCfg(_lib.GEMM_K128, waves, depth, ks, strips))
            for waves in (4, 8):
                for kc in (2, 4, 8):  # shared-activation kernel: chunks per K slice; ksplit follows
                    cfgs.append(_lib.GemmCfg(_lib.GEMM_XS, waves, kc, -(-(k // 128) // kc), 1))
            for waves in (8, 16):
                for depth in (2, 4):
                    for kpw in (1, 2, 4):  # register-resident kernel: chunks per wave; ksplit follows
                        cfgs.append(_lib.GemmCfg(_lib.GEMM_XR, waves, depth, -(-(k // 128) // (waves * kpw)), kpw))
            cfgs = [c for c in cfgs if c.kernel in kern]
            for cfg in cfgs:
                wsz = L.nf4_gemm_workspace_bytes_cfg(M, n, k, ctypes.byref(cfg))
                work = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=dev)
                probe = L.nf4_gemm_ref_cfg(x.data_ptr(), M, ws[0][0].data_ptr(), ws[0][0].numel(),
                                           ws[0][1].data_ptr(), ws[0][1].numel(), ws[0][2].data_ptr(),
                                           ws[0][2].numel(), y.data_ptr(), _lib.BF16, n, k, work.data_ptr(), wsz,
                                           ctypes.byref(cfg), torch.cuda.current_stream().cuda_stream)
                if probe in (_lib.ERR_ARG, _lib.ERR_TOO_LARGE):  # not valid / not fitting at this shape
                    continue
                assert probe == 0, probe

                def run(cfg=cfg, work=work, wsz=wsz):
                    sp = torch.cuda.current_stream().cuda_stream
                    for (q, a1, a2) in ws:
                        rc = L.nf4_gemm_ref_cfg(x.data_ptr(), M, q.data_ptr(), q.numel(), a1.data_ptr(),
                                                a1.numel(), a2.data_ptr(), a2.numel(), y.data_ptr(),
                                                _lib.BF16, n, k, work.data_ptr(), wsz, ctypes.byref(cfg), sp)
                        assert rc == 0, rc

                us = graph_us(run, copies)
                out = y.float()
                if ref is None:
                    ref = out.clone()
                err = float(((out - ref).abs() / (ref.abs() + 1e-2)).max())
                res.append({"cfg": [cfg.kernel, cfg.waves, cfg.depth, cfg.ksplit, cfg.strips], "us": round(us, 2),
                            "TBps": round(wbytes / us / 1e6, 3), "relerr": round(err, 4)})
            # default
            wsz = L.nf4_gemm_workspace_bytes(M, n, k)
            work = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=dev)

            def run_def():
                sp = torch.cuda.current_stream().cuda_stream
                for (q, a1, a2) in ws:
                    assert L.nf4_gemm_ref(x.data_ptr(), M, q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(),
                                          a2.data_ptr(), a2.numel(), y.data_ptr(), _lib.BF16, n, k,
                                          work.data_ptr(), wsz, sp) == 0

            dus = graph_us(run_def, copies)
            res.sort(key=lambda r: r["us"])
            print(json.dumps({"N": n, "K": k, "M": M, "copies": copies, "default_us": round(dus, 2),
                              "default_TBps": round(wbytes / dus / 1e6, 3), "best": res[:8],
                              "worst": res[-2:], "all": res}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
