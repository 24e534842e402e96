"""Per-wave phase timing of the fused-GEMM kernels (diagnostic build `make -C tools gstamps`).

    python tools/gemm_stamps.py --shape 14336,4096 --m 32 [--cfg 5,8,2,2,2 ...]

Each wave stamps s_memrealtime (100 MHz) at the hooks of nf4_gemm.hip (see
tools/gemm_stamps.hip for the slots); prints, per configuration (default: the
library's choice), the launch-wide distribution in us (0/10/50/90/100th
percentiles over waves and launches): wave start spread, prologue (entry ->
prologue barrier), first strip (barrier -> first strip consumed: x and the first
weights arriving), strip loop, the in-loop partial-tile stores + barriers and
reducer sums (summed per wave), final barrier, result stores, split-K hand-off,
and the launch span (first entry -> last exit).  Each launch runs alone on a
weight that is not in any cache (rotating copies), so the span includes the first
loads' latency; the stamps cost a few percent (shares, not absolute speed).
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
# --variant <part>: a stamped ablation build (tools/Makefile libnf4dq_gstamps_<part>.so,
# e.g. skeleton); parsed before the library is imported, since the import loads it
_VAR = next((sys.argv[i + 1] for i, a in enumerate(sys.argv[:-1]) if a == "--variant"), "")
os.environ["NF4DQ_LIB_PATH"] = os.path.join(REPO, "tools", "_build",
                                            f"libnf4dq_gstamps_{_VAR}.so" if _VAR else "libnf4dq_gstamps.so")
from nf4_triton_dequantization_amd import _lib  # noqa: E402


def pct(a):
    a = np.asarray(a, np.float64)
    a = a[~np.isnan(a)]
    if a.size == 0:
        return None
    return [round(float(np.percentile(a, q)), 2) for q in (0, 10, 50, 90, 100)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="14336,4096")
    ap.add_argument("--m", type=int, default=32)
    ap.add_argument("--cfg", action="append", default=[], help="kernel,waves,depth,ksplit,strips (default: library)")
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("--variant", default="", help="stamped ablation build (e.g. skeleton); default: the product")
    ap.add_argument("--chain", type=int, default=1,
                    help="launches back to back per sample (other copies first, no sync between): the stamps "
                         "are the last launch's, in the regime of a decode pass / bench (default 1: alone, cold)")
    args = ap.parse_args()
    L = _lib.lib()
    L.nf4_dbg_set_gemm_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    n, k = (int(v) for v in args.shape.split(","))
    M = args.m
    # distinct copies: a chain's weights stream from HBM, not the 256 MiB Infinity Cache
    copies = max(4, 2 * args.chain, (1024 << 20) // (n * k // 2))
    nb = n * k // 64
    ws = [(torch.randint(0, 256, (n * k // 2,), dtype=torch.uint8, device=dev),
           torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev),
           torch.rand((nb + 255) // 256, device=dev) * 0.01 + 1e-3) for _ in range(copies)]
    x = torch.randn((M, k), device=dev).to(torch.bfloat16)
    y = torch.empty((M, n), dtype=torch.bfloat16, device=dev)
    stamps = torch.zeros(4 << 20, dtype=torch.int64, device=dev)  # 32 MiB: 16 slots x 256 Ki waves
    assert L.nf4_dbg_set_gemm_stamps(stamps.data_ptr()) == 0
    sp = torch.cuda.current_stream().cuda_stream
    for cs in (args.cfg or [None]):
        cfg = _lib.GemmCfg(*(int(v) for v in cs.split(","))) if cs else None
        wsz = (L.nf4_gemm_workspace_bytes_cfg(M, n, k, ctypes.byref(cfg)) if cfg else
               L.nf4_gemm_workspace_bytes(M, n, k))
        work = torch.zeros(max(wsz, 1 << 16), dtype=torch.uint8, device=dev)
        rows = {key: [] for key in ("start", "pro", "pro_x_issue", "pro_ring_issue", "pro_tables", "pro_barrier",
                                    "first", "loop", "red_store_barrier", "red_sum", "final_barrier", "store", "handoff",
                                    "end")}
        spans = []
        for it in range(args.launches + 2):
            q, a1, a2 = ws[(it * args.chain) % copies]
            stamps.zero_()
            torch.cuda.synchronize()
            for c in range(args.chain - 1):  # earlier launches of the chain: their stamps are overwritten
                qc, a1c, a2c = ws[(it * args.chain + c + 1) % copies]
                if cfg is not None:
                    rc = L.nf4_gemm_ref_cfg(x.data_ptr(), M, qc.data_ptr(), qc.numel(), a1c.data_ptr(), a1c.numel(),
                                            a2c.data_ptr(), a2c.numel(), y.data_ptr(), _lib.BF16, n, k,
                                            work.data_ptr(), work.numel(), ctypes.byref(cfg), sp)
                else:
                    rc = L.nf4_gemm_ref(x.data_ptr(), M, qc.data_ptr(), qc.numel(), a1c.data_ptr(), a1c.numel(),
                                        a2c.data_ptr(), a2c.numel(), y.data_ptr(), _lib.BF16, n, k,
                                        work.data_ptr(), work.numel(), sp)
                assert rc == 0, rc
            if cfg is not None:
                rc = L.nf4_gemm_ref_cfg(x.data_ptr(), M, q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(),
                                        a2.data_ptr(), a2.numel(), y.data_ptr(), _lib.BF16, n, k, work.data_ptr(),
                                        work.numel(), ctypes.byref(cfg), sp)
            else:
                rc = L.nf4_gemm_ref(x.data_ptr(), M, q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(),
                                    a2.data_ptr(), a2.numel(), y.data_ptr(), _lib.BF16, n, k, work.data_ptr(),
                                    work.numel(), sp)
            assert rc == 0, rc
            torch.cuda.synchronize()
            if it < 2:
                continue
            st = stamps.view(-1, 16).cpu().numpy().astype(np.float64)
            st = st[st[:, 0] > 0]
            t = st / 100.0  # us (100 MHz)
            t0 = t[:, 0].min()

            def col(i):
                v = t[:, i].copy()
                v[st[:, i] == 0] = np.nan
                return v
            s0, s1, s2, s3, s4, s5, s9, s10, s11, s12 = (col(i) for i in (0, 1, 2, 3, 4, 5, 9, 10, 11, 12))
            s9 = np.where(np.isnan(s9), s5, s9)  # one-slice launches return after their y stores
            rows["start"].append(s0 - t0)
            rows["pro"].append(s1 - s0)
            rows["pro_x_issue"].append(s11 - s0)
            rows["pro_ring_issue"].append(s10 - s11)
            rows["pro_tables"].append(s12 - s10)
            rows["pro_barrier"].append(s1 - s12)
            rows["first"].append(s2 - s1)
            rows["loop"].append(s3 - s1)
            rows["red_store_barrier"].append(st[:, 7] / 100.0)
            rows["red_sum"].append(st[:, 8] / 100.0)
            rows["final_barrier"].append(s4 - s3)
            rows["store"].append(s5 - s4)
            rows["handoff"].append(s9 - s5)
            rows["end"].append(s9 - t0)
            spans.append(np.nanmax(s9) - t0)
        out = {"variant": args.variant or "product", "chain": args.chain, "cfg": cs or "library", "N": n, "K": k, "M": M, "waves_per_launch": int(len(rows["start"][0])),
               "span_us": pct(spans)}
        for key, v in rows.items():
            out[key] = pct(np.concatenate(v))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
