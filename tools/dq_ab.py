"""Interleaved A/B of dequant launch configurations (one process, one box).

    python tools/dq_ab.py [--shapes 4096x4096,8192x8192] [--flags 0,0xE00,0x6E00] [--rounds 7]

Per shape: rotating buffer sets of >= 1 GiB (each with its own absmax / nested
absmax, as real weights), every set touched once; then `rounds` rounds, each
timing every configuration in turn as bench.py does (device spin covering the
host's submission, 8 untimed lead launches, K launches between HIP events on the
launch stream).  Prints one JSON line per (shape, flags): median and spread of the
per-launch time over rounds, and the fraction of the 8 TB/s peak (SURVEY §8d
bytes).  Interleaving puts box drift into every configuration alike, so
differences of ~1 % resolve (separate processes differ by ~3 %).
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

PEAK = 8e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096x4096,8192x8192")
    ap.add_argument("--flags", default="0,0xE00,0x6E00")
    ap.add_argument("--bpcu", default="0")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--sets", default="0", help="buffer-set counts to try (0 = enough for 1 GiB)")
    ap.add_argument("--pad-kb", default="0", help="KiB allocated between the arrays of a set (placement probe)")
    ap.add_argument("--pool", default="0", help="1 = every array a 2 MiB-aligned slice of ONE allocation (0,1 = both)")
    args = ap.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    torch.cuda._sleep(2_000_000)
    e1.record(st)
    torch.cuda.synchronize()
    cyc_per_us = 2_000_000 / max(e0.elapsed_time(e1) * 1e3, 1.0)
    cfgs = [(int(b), int(f, 0)) for f in args.flags.split(",") for b in args.bpcu.split(",")]
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    todo = [(shp, int(sv), int(pk), int(pl)) for shp in args.shapes.split(",") for sv in args.sets.split(",")
            for pk in args.pad_kb.split(",") for pl in args.pool.split(",")]
    for shp, sets_req, pad_kb, pool in todo:
        m, n = (int(v) for v in shp.split("x"))
        nbytes, nb = m * n // 2, m * n // 64
        n2 = (nb + 255) // 256
        alg = nbytes + 2 * m * n + nb + 4 * n2
        P = sets_req or max(2, -(-(1 << 30) // (nbytes * 5)))
        pads = []

        def pad():
            if pad_kb:
                pads.append(torch.empty(pad_kb << 10, dtype=torch.uint8, device=dev))
        sets = []
        big = None
        if pool:
            al = 2 << 20
            per = [nbytes, nb, 4 * n2, 2 * m * n]
            per = [(b + al - 1) // al * al for b in per]
            big = torch.empty(P * sum(per) + al, dtype=torch.uint8, device=dev)
            off = (-big.data_ptr()) % al
        for _ in range(P):
            if pool:
                views = []
                for b in per:
                    views.append(big[off:off + b])
                    off += b
                q = views[0][:nbytes]
                q.copy_(torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev, generator=gen))
                a1 = views[1][:nb]
                a1.copy_(torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=gen))
                a2 = views[2][:4 * n2].view(torch.float32)
                a2.copy_(torch.rand(n2, device=dev, generator=gen) * 0.01 + 1e-3)
                sets.append((q, a1, a2, views[3][:2 * m * n].view(torch.bfloat16).view(m, n)))
                continue
            q = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev, generator=gen)
            pad()
            a1 = torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=gen)
            a2 = torch.rand(n2, device=dev, generator=gen) * 0.01 + 1e-3
            pad()
            sets.append((q, a1, a2, torch.empty((m, n), dtype=torch.bfloat16, device=dev)))
        layout = [[(t.data_ptr() - sets[0][0].data_ptr()) >> 10 for t in s_] for s_ in sets[:2]]
        cobj = {c: _lib.LaunchCfg(4, c[0], 1, c[1]) for c in cfgs}

        def launch(i, c):
            q, a1, a2, o = sets[i % P]
            rc = L.nf4_dequant_ref_cfg(q.data_ptr(), nbytes, a1.data_ptr(), nb, a2.data_ptr(), n2, o.data_ptr(),
                                       _lib.BF16, m, n, ctypes.byref(cobj[c]), st.cuda_stream)
            assert rc == 0, rc

        for c in cfgs:
            for i in range(P):
                launch(i, c)
        torch.cuda.synchronize()
        res = {c: [] for c in cfgs}
        for _ in range(args.rounds):
            for c in cfgs:
                torch.cuda._sleep(int(cyc_per_us * (40.0 * (args.steps + 8) + 200.0)))
                for j in range(8):
                    launch(j - 8, c)
                e0.record(st)
                for i in range(args.steps):
                    launch(i, c)
                e1.record(st)
                torch.cuda.synchronize()
                res[c].append(e0.elapsed_time(e1) * 1e3 / args.steps)
        for c in cfgs:
            ts = sorted(res[c])
            med = ts[len(ts) // 2]
            print(json.dumps({"m": m, "n": n, "blocks_per_cu": c[0], "flags": hex(c[1]), "sets": P, "pad_kb": pad_kb,
                              "pool": pool, "footprint_MB": round(P * (nbytes * 5 + nb) / 1e6),
                              "offsets_kb": layout,
                              "us_median": round(med, 3), "us_min": round(ts[0], 3), "us_max": round(ts[-1], 3),
                              "frac": round(alg / (med * 1e-6) / PEAK, 4)}), flush=True)
        del sets, pads, big
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
