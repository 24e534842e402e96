"""Launch-config sweep for nf4_flat_kernel (interleaved rounds in one process, rule 24).

    python tools/tune.py [--m 4096 --n 4096 --dtype bf16 --rounds 5]

For each config: mean per-launch kernel time from HIP events (launches queued
behind a spin kernel), and graph-replay time per step (back-to-back launches
over rotating buffer sets).  Prints one JSON line per config (median over rounds).
"""
from __future__ import annotations

import argparse
import ctypes
import itertools
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from nf4_triton_dequantization_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--sets", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=64)
    ap.add_argument("--tiles", default="4")
    ap.add_argument("--bpcu", default="0,1,2,4,8")
    ap.add_argument("--nt", default="1")
    ap.add_argument("--flags", default="0", help="nf4_launch_cfg.flags: reserved, must be 0 (kept for old logs)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    m, n, P = args.m, args.n, args.sets
    dt = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}[args.dtype]
    code = {"bf16": _lib.BF16, "f16": _lib.F16, "f32": _lib.F32}[args.dtype]
    nb = m * n // 64
    n2 = (nb + 255) // 256
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    sets = []
    for _ in range(P):
        q = torch.randint(0, 256, (m * n // 2,), dtype=torch.uint8, device=dev, generator=g)
        a1 = torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
        a2 = torch.rand(n2, device=dev, generator=g) * 0.01
        sets.append((q, a1, a2, torch.empty((m, n), dtype=dt, device=dev)))
    L = _lib.lib()
    out_b = torch.empty((), dtype=dt).element_size()
    alg = m * n // 2 + m * n * out_b + nb + 4 * min(n2, m * (((n + 63) // 64 + 3) // 4))

    cfgs = [c for c in itertools.product([int(x) for x in args.tiles.split(",")],
                                         [int(x) for x in args.bpcu.split(",")],
                                         [int(x) for x in args.nt.split(",")],
                                         [int(x, 0) for x in args.flags.split(",")])]

    def launch(i, cfg, sp):
        q, a1, a2, out = sets[i % P]
        rc = L.nf4_dequant_ref_cfg(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                   out.data_ptr(), code, m, n, ctypes.byref(cfg), sp)
        assert rc == 0, rc

    stream = torch.cuda.current_stream()
    ok = []
    for c in cfgs:  # drop combinations the ABI rejects (NF4DQ_ERR_ARG)
        q, a1, a2, out = sets[0]
        rc = L.nf4_dequant_ref_cfg(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                   out.data_ptr(), code, m, n, ctypes.byref(_lib.LaunchCfg(*c)),
                                   stream.cuda_stream)
        if rc == 0:
            ok.append(c)
    cfgs = ok
    res = {c: {"ev": [], "graph": []} for c in cfgs}
    graphs = {}
    for c in cfgs:
        cfg = _lib.LaunchCfg(*c)
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph):
            sp = torch.cuda.current_stream().cuda_stream
            for i in range(args.launches):
                launch(i, cfg, sp)
        graphs[c] = (gph, cfg)
    for r in range(args.rounds):
        for c in cfgs:
            gph, cfg = graphs[c]
            R = args.launches
            st = [torch.cuda.Event(enable_timing=True) for _ in range(R)]
            en = [torch.cuda.Event(enable_timing=True) for _ in range(R)]
            torch.cuda.synchronize()
            torch.cuda._sleep(20_000_000)
            for i in range(R):
                st[i].record(stream)
                launch(i, cfg, stream.cuda_stream)
                en[i].record(stream)
            torch.cuda.synchronize()
            res[c]["ev"].append(float(np.mean([a.elapsed_time(b) for a, b in zip(st, en)]) * 1e3))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            gph.replay()
            torch.cuda.synchronize()
            e0.record(stream)
            gph.replay()
            e1.record(stream)
            torch.cuda.synchronize()
            res[c]["graph"].append(e0.elapsed_time(e1) * 1e3 / R)
    for c in cfgs:
        ev = float(np.median(res[c]["ev"]))
        gr = float(np.median(res[c]["graph"]))
        print(json.dumps({"tile_dwords": c[0], "blocks_per_cu": c[1], "nt": c[2], "flags": c[3],
                          "kernel_us_events": round(ev, 3),
                          "graph_us_per_step": round(gr, 3), "GBps_events": round(alg / ev / 1e3, 1),
                          "GBps_graph": round(alg / gr / 1e3, 1), "m": m, "n": n, "dtype": args.dtype}), flush=True)


if __name__ == "__main__":
    main()
