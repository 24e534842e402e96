"""Per-launch time of the fused decode GEMM (library choice), graph replay vs eager.

    [NF4DQ_LIB_PATH=tools/_build/libnf4dq_<x>.so] python tools/gemm_ab.py [--ms 1,16,32]
        [--shapes 14336,4096;4096,4096;4096,14336] [--label name] [--cfgs "default;6,8,0,1,0"]

Each shape streams `copies` distinct weights (> the 256 MiB Infinity Cache) in
turn.  ``graph``: the launches captured once, median of 5 replays (what
tools/sweep_gemm.py and tools/bench_gemm.py report); ``eager``: a device spin
that covers the host's submission, then the same launches between HIP events on
the launch stream (what bench.py does for the dequant).  One JSON line per
(shape, M, cfg).  ``--cfgs``: decompositions timed in turn on the same weights
("default" = the library's choice through nf4_gemm_ref, else kernel,waves,depth,
ksplit,strips through nf4_gemm_ref_cfg; one that the ABI rejects is skipped).
Run once per library build for an A/B on one box.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,16,32")
    ap.add_argument("--shapes", default="14336,4096;4096,4096;4096,14336")
    ap.add_argument("--budget-mb", type=int, default=768)
    ap.add_argument("--label", default=os.path.basename(os.environ.get("NF4DQ_LIB_PATH", "prod")))
    ap.add_argument("--cfgs", default="default")
    args = ap.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    torch.cuda._sleep(2_000_000)
    e1.record(st)
    torch.cuda.synchronize()
    cyc_per_us = 2_000_000 / max(e0.elapsed_time(e1) * 1e3, 1.0)
    for sh in args.shapes.split(";"):
        n, k = (int(v) for v in sh.split(","))
        copies = max(8, args.budget_mb * (1 << 20) // (n * k // 2))
        nb = n * k // 64
        ws = [(torch.randint(0, 256, (n * k // 2,), dtype=torch.uint8, device=dev, generator=gen),
               torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=gen),
               torch.rand((nb + 255) // 256, device=dev, generator=gen) * 0.01 + 1e-3) for _ in range(copies)]
        for M in (int(v) for v in args.ms.split(",")):
            x = torch.randn((M, k), device=dev, generator=gen).to(torch.bfloat16)
            y = torch.empty((M, n), dtype=torch.bfloat16, device=dev)
            for cs in args.cfgs.split(";"):
                cfg = None if cs == "default" else _lib.GemmCfg(*(int(v) for v in cs.split(",")))
                one(L, M, n, k, x, y, ws, copies, cfg, cs, st, e0, e1, cyc_per_us, args.label)


def one(L, M, n, k, x, y, ws, copies, cfg, cs, st, e0, e1, cyc_per_us, label):
    dev = x.device
    if cfg is None:
        wsz = L.nf4_gemm_workspace_bytes(M, n, k)
    else:
        wsz = L.nf4_gemm_workspace_bytes_cfg(M, n, k, ctypes.byref(cfg))
    work = torch.zeros(max(wsz, 1 << 16), dtype=torch.uint8, device=dev)

    def call(i):
        q, a1, a2 = ws[i % copies]
        a = (x.data_ptr(), M, q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
             y.data_ptr(), _lib.BF16, n, k, work.data_ptr(), work.numel())
        if cfg is None:
            return L.nf4_gemm_ref(*a, torch.cuda.current_stream().cuda_stream)
        return L.nf4_gemm_ref_cfg(*a, ctypes.byref(cfg), torch.cuda.current_stream().cuda_stream)

    rc = call(0)
    if rc:
        print(json.dumps({"lib": label, "N": n, "K": k, "M": M, "cfg": cs, "skipped": _lib.strerror(rc)}), flush=True)
        return

    def launch(i):
        rc = call(i)
        assert rc == 0, rc

    for i in range(copies):
        launch(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(copies):
            launch(i)
    g.replay()
    torch.cuda.synchronize()
    tg, te = [], []
    for _ in range(5):
        e0.record(st)
        g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        tg.append(e0.elapsed_time(e1) * 1e3 / copies)
        torch.cuda._sleep(int(cyc_per_us * (40.0 * copies + 200.0)))
        e0.record(st)
        for i in range(copies):
            launch(i)
        e1.record(st)
        torch.cuda.synchronize()
        te.append(e0.elapsed_time(e1) * 1e3 / copies)
    tg.sort()
    te.sort()
    if wsz:
        assert L.nf4_gemm_check_workspace(work.data_ptr(), wsz, st.cuda_stream) == 0
    print(json.dumps({"lib": label, "N": n, "K": k, "M": M, "cfg": cs, "copies": copies,
                      "graph_us": round(tg[2], 3), "eager_us": round(te[2], 3),
                      "eager_min_us": round(te[0], 3)}), flush=True)
    del g


if __name__ == "__main__":
    main()
