"""Time chosen fused-GEMM configs against the diagnostic library variants.

    python tools/gemm_probe.py --lib {prod,dbg1,dbg2} --shape N,K --m M --cfg k,w,d,ks,t [--cfg ...]

dbg1 = loads only, dbg2 = dequant/MMA body only (tools/Makefile `dbg`).
Prints us per launch (hipGraph of `copies` distinct weights, > MALL).
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
from sweep_gemm import graph_us  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="prod")
    ap.add_argument("--shape", action="append", default=[])
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--cfg", action="append", default=[])
    ap.add_argument("--budget-mb", type=int, default=768)
    args = ap.parse_args()
    if args.lib != "prod":
        _lib.LIB_PATH = os.path.join(REPO, "tools", "_build", f"libnf4dq_{args.lib}.so")
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    for sh in args.shape or ["14336,4096"]:
        n, k = (int(v) for v in sh.split(","))
        copies = max(8, args.budget_mb * (1 << 20) // (n * k // 2))
        nb = n * k // 64
        ws = [(torch.randint(0, 256, (n * k // 2,), dtype=torch.uint8, device=dev, generator=gen),
               torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=gen),
               torch.rand((nb + 255) // 256, device=dev, generator=gen) * 0.01 + 1e-3) for _ in range(copies)]
        wbytes = n * k // 2 + nb + 4 * ((nb + 255) // 256)
        M = args.m
        x = torch.randn((M, k), device=dev).to(torch.bfloat16)
        y = torch.empty((M, n), dtype=torch.bfloat16, device=dev)
        for cs in args.cfg:
            cfg = _lib.GemmCfg(*(int(v) for v in cs.split(",")))
            wsz = L.nf4_gemm_workspace_bytes_cfg(M, n, k, ctypes.byref(cfg))
            work = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=dev)
            q0, a10, a20 = ws[0]
            rc0 = L.nf4_gemm_ref_cfg(x.data_ptr(), M, q0.data_ptr(), q0.numel(), a10.data_ptr(), a10.numel(),
                                     a20.data_ptr(), a20.numel(), y.data_ptr(), _lib.BF16, n, k, work.data_ptr(), wsz,
                                     ctypes.byref(cfg), torch.cuda.current_stream().cuda_stream)
            if rc0 != 0:  # not a valid decomposition for this shape
                print(json.dumps({"lib": args.lib, "N": n, "K": k, "M": M, "cfg": cs, "rc": rc0}), flush=True)
                continue

            def run(cfg=cfg, work=work, wsz=wsz):
                sp = torch.cuda.current_stream().cuda_stream
                for (q, a1, a2) in ws:
                    rc = L.nf4_gemm_ref_cfg(x.data_ptr(), M, q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(),
                                            a2.data_ptr(), a2.numel(), y.data_ptr(), _lib.BF16, n, k,
                                            work.data_ptr(), wsz, ctypes.byref(cfg), sp)
                    assert rc == 0, rc

            us = graph_us(run, copies)
            print(json.dumps({"lib": args.lib, "N": n, "K": k, "M": M, "cfg": cs, "us": round(us, 2),
                              "TBps": round(wbytes / us / 1e6, 3)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
