"""Per-wave phase timing of the streaming GEMM kernel (diagnostic build dbg3).

    python tools/gemm_stamps.py --shape 14336,4096 --m 1 --cfg 2,4,2,1,2 [--cfg ...]

Each wave stamps s_memrealtime (100 MHz) at start, after its workgroup's
prologue barrier, after its chunk loop, and at its end; prints the launch-wide
distribution (us): wave start spread, prologue, loop, epilogue, and the
kernel span (first start -> last end).  Shares, not absolute speed: the
stamps fence overlaps the product build has.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from nf4_triton_dequantization_amd import _lib  # noqa: E402


def pct(a):
    return [round(float(np.percentile(a, q)), 2) for q in (0, 10, 50, 90, 100)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="14336,4096")
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--cfg", action="append", default=[])
    args = ap.parse_args()
    _lib.LIB_PATH = os.path.join(REPO, "tools", "_build", "libnf4dq_dbg3.so")
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    n, k = (int(v) for v in args.shape.split(","))
    M = args.m
    copies = max(4, (512 << 20) // (n * k // 2))
    nb = n * k // 64
    ws = [(torch.randint(0, 256, (n * k // 2,), dtype=torch.uint8, device=dev),
           torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev),
           torch.rand((nb + 255) // 256, device=dev) * 0.01 + 1e-3) for _ in range(copies)]
    x = torch.randn((M, k), device=dev).to(torch.bfloat16)
    y = torch.empty((M, n), dtype=torch.bfloat16, device=dev)
    work = torch.zeros((64 << 10) + (8 << 20), dtype=torch.uint8, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    for cs in args.cfg:
        cfg = _lib.GemmCfg(*(int(v) for v in cs.split(",")))
        waves_total = (n // (16 * cfg.strips)) * cfg.waves
        spans, rows = [], []
        for it in range(copies):
            q, a1, a2 = ws[it]
            work[64 << 10:].zero_()
            rc = L.nf4_gemm_ref_cfg(x.data_ptr(), M, q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(),
                                    a2.data_ptr(), a2.numel(), y.data_ptr(), _lib.BF16, n, k, work.data_ptr(),
                                    work.numel(), ctypes.byref(cfg), sp)
            assert rc == 0, rc
            torch.cuda.synchronize()
            if it < 2:
                continue
            st = work[64 << 10:].view(torch.int64)[: waves_total * 8].cpu().numpy().reshape(-1, 8)
            t = st[:, :4].astype(np.float64) / 100.0  # us
            t0 = t[:, 0].min()
            rows.append({"start": t[:, 0] - t0, "pro": t[:, 1] - t[:, 0], "loop": t[:, 2] - t[:, 1],
                         "epi": np.where(t[:, 3] > 0, t[:, 3] - t[:, 2], np.nan), "end": t[:, 3] - t0})
            spans.append(np.nanmax(np.where(t[:, 3] > 0, t[:, 3], t[:, 2])) - t0)
        agg = {kk: np.concatenate([r[kk] for r in rows]) for kk in rows[0]}
        print(json.dumps({"cfg": cs, "N": n, "K": k, "M": M, "span_us": pct(spans),
                          "start": pct(agg["start"]), "prologue": pct(agg["pro"]), "loop": pct(agg["loop"]),
                          "epilogue": pct(agg["epi"][~np.isnan(agg["epi"])]),
                          "end": pct(agg["end"][~np.isnan(agg["end"])])}), flush=True)


if __name__ == "__main__":
    main()
