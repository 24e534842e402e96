"""Where do the headline's reads come from?  Independent input / output rotation A/B.

    python tools/cache_ab.py [--shape 4096x4096] [--dtype bf16|f32]
                             [--pairs 13x13,40x13,13x60@4,...] [--rounds 5] [--steps 128]

Step i of a configuration ``IxO`` reads input set ``i % I`` (packed weight + absmax +
nested absmax) and writes output set ``i % O``, so the distinct *read* bytes
(I x 8.65 MB at 4096^2) and the distinct *written* bytes (O x 33.5 MB bf16) of the
rotation are set independently.  If a configuration with many input sets and few
output sets is slow while the converse is fast, the per-launch time depends on
whether the packed weights stay in the 256 MiB Infinity Cache (the nt output stores
not displacing them); if the converse holds, on how much address space the
rotation walks (translation reach).  VERDICT r03 "Next round" item 1.
``IxO@b`` times launch configuration blocks_per_cu = b (nf4_dequant_ref_cfg; the
library default, b = 0, otherwise): the launch knobs re-checked in the regime
where the weights stream from HBM.  ``--libs a.so,b.so``: every configuration is
also timed through each of these builds of the C ABI (tools/dq_variants.hip A/B
libraries), loaded side by side in this process and interleaved with the product.

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
    ap.add_argument("--libs", default="", help="extra builds of the C ABI to time beside the product")
    args = ap.parse_args()
    libs = [("prod", _lib.lib())]
    for path in [v for v in args.libs.split(",") if v]:
        h = ctypes.CDLL(os.path.abspath(path))
        for name, (res_t, argt) in _lib.SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res_t, argt
        libs.append((os.path.basename(path).replace("libnf4dq_", "").replace(".so", ""), h))
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
    pairs = []
    for p in args.pairs.split(","):
        io, _, b = p.partition("@")
        for li in range(len(libs)):
            pairs.append(tuple(int(v) for v in io.split("x")) + (int(b or 0), li))
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

    cfgs = {b: _lib.LaunchCfg(4, b, 1, 0) for b in {p[2] for p in pairs}}

    def launch(i, I, O, b=0, li=0):
        L = libs[li][1]
        q, a1, a2 = ins[i % I]
        if b:
            rc = L.nf4_dequant_ref_cfg(q.data_ptr(), nbytes, a1.data_ptr(), nb, a2.data_ptr(), n2,
                                       outs[i % O].data_ptr(), code, m, n, ctypes.byref(cfgs[b]), sp)
        else:
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
    for li in range(len(libs)):
        for i in range(max(I_max, O_max)):
            launch(i, I_max, O_max, 0, li)
    torch.cuda.synchronize()
    res = {p: [] for p in pairs}
    for _ in range(args.rounds):
        for (I, O, b, li) in pairs:
            for i in range(max(I, O)):  # the configuration's own untimed pass
                launch(i, I, O, b, li)
            torch.cuda._sleep(int(cyc_per_us * (30.0 * (args.steps + args.lead) + 200.0)))
            for j in range(args.lead):
                launch(j - args.lead + 10 * I * O, I, O, b, li)
            e0.record(st)
            for i in range(args.steps):
                launch(i, I, O, b, li)
            e1.record(st)
            torch.cuda.synchronize()
            res[(I, O, b, li)].append(e0.elapsed_time(e1) * 1e3 / args.steps)
    # hygiene: set 0's output vs the oracle (first 32 rows)
    import nf4_oracle as Ora

    r = 32
    oks = []
    for li in range(len(libs)):
        outs[0].zero_()
        launch(0, 1, 1, 0, li)
        torch.cuda.synchronize()
        if args.dtype != "f32":
            want = Ora.dequant_ref_np(p0[: r * n // 2], a10, a20, r, n, Ora.BF16 if args.dtype == "bf16" else Ora.F16)
            got = outs[0][:r].contiguous().view(torch.int16).cpu().numpy().view(np.uint16)
            oks.append(bool(np.array_equal(got, want)))
        else:
            oks.append(None)
    for (I, O, b, li) in pairs:
        ok = oks[li]
        ts = sorted(res[(I, O, b, li)])
        med = ts[len(ts) // 2]
        rd = I * (nbytes + nb + 4 * n2)
        wr = O * m * n * ob
        print(json.dumps({"tag": args.tag, "m": m, "n": n, "dtype": args.dtype, "in_sets": I, "out_sets": O,
                          "blocks_per_cu": b, "lib": libs[li][0],
                          "read_MB": round(rd / 1e6, 1), "written_MB": round(wr / 1e6, 1),
                          "footprint_MB": round((rd + wr) / 1e6, 1),
                          "us_median": round(med, 3), "us_min": round(ts[0], 3), "us_max": round(ts[-1], 3),
                          "frac": round(alg / (med * 1e-6) / PEAK, 4), "steps": args.steps,
                          "rounds": args.rounds, "checked": ok}), flush=True)


if __name__ == "__main__":
    main()
