"""Run every decomposition the tuning ABI accepts for one GEMM shape, one launch at a
time, printing each config (flushed) before it runs -- to name the config behind a
GPU failure.  Diagnostic only.

    python tools/cfg_isolate.py --m 1 --n 256 --k 4096 [--kernels 3,2,1]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from nf4_triton_dequantization_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--kernels", default="3")
    a = ap.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    M, N, K = a.m, a.n, a.k
    nb = N * K // 64
    q = torch.randint(0, 256, (N * K // 2,), dtype=torch.uint8, device=dev, generator=g)
    a1 = torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
    a2 = torch.rand(((nb + 255) // 256,), device=dev, generator=g) + 0.01
    x = torch.randn((M, K), device=dev, generator=g).to(torch.bfloat16)
    y = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    for kernel in (int(v) for v in a.kernels.split(",")):
        for waves in (4, 8, 16):
            for depth in (1, 2, 4, 8):
                for strips in (1, 2, 4):
                    for ks in (1, 2, 3):
                        cfg = _lib.GemmCfg(kernel, waves, depth, ks, strips)
                        wsz = L.nf4_gemm_workspace_bytes_cfg(M, N, K, ctypes.byref(cfg))
                        ws = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=dev)
                        torch.cuda.synchronize()
                        print("cfg", kernel, waves, depth, strips, ks, "ws", wsz, file=sys.stderr, flush=True)
                        rc = L.nf4_gemm_ref_cfg(x.data_ptr(), M, q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(),
                                                a2.data_ptr(), a2.numel(), y.data_ptr(), _lib.BF16, N, K,
                                                ws.data_ptr(), wsz, ctypes.byref(cfg),
                                                torch.cuda.current_stream().cuda_stream)
                        torch.cuda.synchronize()
                        print("  rc", rc, file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
