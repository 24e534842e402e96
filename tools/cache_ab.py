"""Where do the headline's reads come from?  Independent input / output rotation A/B.

    python tools/cache_ab.py [--shape 4096x4096] [--dtype bf16|f32]
                             [--pairs 13x13,40x13,13x60,...] [--rounds 5] [--steps 128]

Step i of a configuration ``IxO`` reads input set ``i % I`` (packed weight + absmax +
nested absmax) and writes output set ``i % O``, so the distinct *read* bytes
(I x 8.65 MB at 4096^2) and the distinct *written* bytes (O x 33.5 MB bf16) of the
rotation are set independently.  If a configuration with many input sets and few
output sets is slow while the converse is fast, the per-launch time depends on
whether the packed weights stay in the 256 MiB Infinity Cache (the nt output stores
not displacing them); if the converse holds, on how much address space the
rotation walks (translation reach).  VERDICT r03 "Next round" item 1.

Timing as bench.py: one untimed pass over every set of a configuration, a device
spin covering the host's submission, 16 untimed lead launches, K eager launches
of the product entry ``nf4_dequant_ref`` between HIP events on the launch stream.
The configurations are interleaved round by round so box drift hits them alike.
Each line: per-launch median / min / max over rounds and the fraction of 8 TB/s
(SURVEY §8d algorithmic bytes).  Outputs of the last launch of set 0 are checked
against the C oracle on their first 32 rows (measurement hygiene, not a test).
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
sys.path.insert(0, os.path.join(REPO, "oracle"))
import workloads as W  # noqa: E402
from nf4_triton_dequantization_amd import _lib  # noqa: E402

PEAK = 8e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4096x4096")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "f32"])
    ap.add_argument("--pairs", default="13x13,40x13,13x60,2x2,60x60")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--lead", type=int, default=16)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = torch.cuda.current_stream()
    m, n = (int(v) for v in args.shape.split("x"))
    code = {"bf16": _lib.BF16, "f16": _lib.F16, "f32": _lib.F32}[args.dtype]
    tdt = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}[args.dtype]
    ob = 4 if args.dtype == "f32" else 2
    nbytes, nb = m * n // 2, m * n // 64
    n2 = (nb + 255) // 256
    alg = W.algorithmic_bytes(m, n, ob, nb, n2)
    pairs = [tuple(int(v) for v in p.split("x")) for p in args.pairs.split(",")]
    I_max = max(p[0] for p in pairs)
    O_max = max(p[1] for p in pairs)

    # inputs: one host generation, I_max device copies (distinct addresses are what
    # keep a set out of the caches); outputs: O_max separate allocations
    p0, a10, a20 = W.make_inputs(m, n, 3409)
    q0, a1_0, a2_0 = (torch.from_numpy(p0).to(dev), torch.from_numpy(a10).to(dev), torch.from_numpy(a20).to(dev))
    ins = [(q0, a1_0, a2_0)] + [(q0.clone(), a1_0.clone(), a2_0.clone()) for _ in range(I_max - 1)]
    outs = [torch.empty((m, n), dtype=tdt, device=dev) for _ in range(O_max)]
    torch.cuda.synchronize()

    sp = st.cuda_stream

    def launch(i, I, O):
        q, a1, a2 = ins[i % I]
        rc = L.nf4_dequant_ref(q.data_ptr(), nbytes, a1.data_ptr(), nb, a2.data_ptr(), n2,
                               outs[i % O].data_ptr(), code, m, n, sp)
        if rc:
            raise RuntimeError(_lib.strerror(rc))

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    torch.cuda._sleep(2_000_000)
    e1.record(st)
    torch.cuda.synchronize()
    cyc_per_us = 2_000_000 / max(e0.elapsed_time(e1) * 1e3, 1.0)

    # touch every set once (TLB-warm, as resident weights are)
    for i in range(max(I_max, O_max)):
        launch(i, I_max, O_max)
    torch.cuda.synchronize()
    res = {p: [] for p in pairs}
    for _ in range(args.rounds):
        for (I, O) in pairs:
            for i in range(max(I, O)):  # the configuration's own untimed pass
                launch(i, I, O)
            torch.cuda._sleep(int(cyc_per_us * (30.0 * (args.steps + args.lead) + 200.0)))
            for j in range(args.lead):
                launch(j - args.lead + 10 * I * O, I, O)
            e0.record(st)
            for i in range(args.steps):
                launch(i, I, O)
            e1.record(st)
            torch.cuda.synchronize()
            res[(I, O)].append(e0.elapsed_time(e1) * 1e3 / args.steps)
    # hygiene: set 0's output vs the oracle (first 32 rows)
    import nf4_oracle as Ora

    launch(0, 1, 1)
    torch.cuda.synchronize()
    r = 32
    if args.dtype != "f32":
        want = Ora.dequant_ref_np(p0[: r * n // 2], a10, a20, r, n, Ora.BF16 if args.dtype == "bf16" else Ora.F16)
        got = outs[0][:r].contiguous().view(torch.int16).cpu().numpy().view(np.uint16)
        ok = bool(np.array_equal(got, want))
    else:
        ok = None
    for (I, O) in pairs:
        ts = sorted(res[(I, O)])
        med = ts[len(ts) // 2]
        rd = I * (nbytes + nb + 4 * n2)
        wr = O * m * n * ob
        print(json.dumps({"tag": args.tag, "m": m, "n": n, "dtype": args.dtype, "in_sets": I, "out_sets": O,
                          "read_MB": round(rd / 1e6, 1), "written_MB": round(wr / 1e6, 1),
                          "footprint_MB": round((rd + wr) / 1e6, 1),
                          "us_median": round(med, 3), "us_min": round(ts[0], 3), "us_max": round(ts[-1], 3),
                          "frac": round(alg / (med * 1e-6) / PEAK, 4), "steps": args.steps,
                          "rounds": args.rounds, "checked": ok}), flush=True)


if __name__ == "__main__":
    main()
