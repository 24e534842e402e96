"""Memory-system twins of the 4096^2 dequant launch, timed exactly as bench.py times it.

    python tools/stream_probe.py [--shape 4096x4096] [--steps 20,128] [--rounds 7]
                                 [--kernels prod,mix:2:18:1,rd:2:1,wr:18:1,empty] [--libs a.so,...]

Kernels (tools/stream_probe.hip, ``tools/_build/libstreamprobe.so``):
  ``mix:LD:ST:TPW``  the product's loads and stores, no decode (LD/ST = aux policy bits;
                     TPW = adjacent tiles per wave)
  ``rd:LD:TPW``      the product's packed-weight loads only (8.4 MB at 4096^2)
  ``wr:ST:TPW``      the product's output stores only (33.5 MB at 4096^2, bf16-sized)
  ``empty``          the same grid, an empty body (launch + boundary alone)
  ``emptydiv:D``     an empty body on a grid D times smaller; ``empty1`` one workgroup
  ``mixs:ST:CH``     mix with the product's scale gathers and CH dependent VALU ops per
                     stored dword (stand-in for decode latency)
  ``prod``           nf4_dequant_ref (the product, bf16); ``prod16`` the same with fp16 output
  ``bnb``            nf4_dequant_bnb (bitsandbytes semantics, blocksize 64 / nested 256),
                     bf16; ``<lib>@bnb`` the same through a --libs library
  ``<lib>``          nf4_dequant_ref of a library given with --libs (basename without
                     ``libnf4dq_`` / ``.so``); ``<lib>@16`` the same with fp16 output

Timing per configuration and round, as bench.py's timed region: one untimed pass over
every buffer set, a device spin that covers the host's submission, 16 untimed lead
launches of the preceding sets, then K eager launches between HIP events on the launch
stream.  Input sets (packed weight + statistics) and output sets rotate independently
with >= 512 MiB of distinct reads and of distinct writes (the weights stream from HBM,
profiles/r04/cache/).  Configurations are interleaved round by round; each line gives
the median / min / max per-launch time over the rounds for each K, and the fraction of
8 TB/s for the dequant's algorithmic bytes (so every twin reads as "the dequant at
this speed would be ...").
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import workloads as W  # noqa: E402
from nf4_triton_dequantization_amd import _lib  # noqa: E402

PEAK = 8e12
BNB_OFFSET = 0.0123
KIND = {"mix": 0, "rd": 1, "wr": 2, "empty": 3, "emptydiv": 4, "empty1": 5, "mixs": 6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4096x4096")
    ap.add_argument("--steps", default="20,128")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--lead", type=int, default=16)
    ap.add_argument("--kernels", default="prod,mix:2:18:1,rd:2:1,wr:18:1,empty")
    ap.add_argument("--libs", default="")
    ap.add_argument("--tag", default="")
    ap.add_argument("--idle-ms", type=float, default=0.0,
                    help="host sleep with the GPU idle before each configuration's spin (DPM probe)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = torch.cuda.current_stream()
    sp = st.cuda_stream
    m, n = (int(v) for v in args.shape.split("x"))
    nbytes, nb = m * n // 2, m * n // 64
    n2 = (nb + 255) // 256
    alg = W.algorithmic_bytes(m, n, 2, nb, n2)
    P = ctypes.CDLL(os.path.join(REPO, "tools", "_build", "libstreamprobe.so"))
    P.twin_launch.restype = ctypes.c_int
    P.twin_launch.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_void_p]
    libs = {"prod": _lib.lib()}
    for path in [v for v in args.libs.split(",") if v]:
        h = ctypes.CDLL(os.path.abspath(path))
        for name, (res_t, argt) in _lib.SIGNATURES.items():
            fn = getattr(h, name, None)
            if fn is not None:
                fn.restype, fn.argtypes = res_t, argt
        libs[os.path.basename(path).replace("libnf4dq_", "").replace(".so", "")] = h

    read_set = nbytes + nb + 4 * n2
    PI = -(-(512 << 20) // read_set)
    PO = -(-(512 << 20) // (4 * nbytes))
    p0, a10, a20 = W.make_inputs(m, n, 3409)
    q0, a1_0, a2_0 = (torch.from_numpy(p0).to(dev), torch.from_numpy(a10).to(dev), torch.from_numpy(a20).to(dev))
    ins = [(q0, a1_0, a2_0)] + [(q0.clone(), a1_0.clone(), a2_0.clone()) for _ in range(PI - 1)]
    outs = [torch.empty((m, n), dtype=torch.bfloat16, device=dev) for _ in range(PO)]
    sink = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
    # bitsandbytes semantics (spec "bnb" / "<lib>@bnb"): the nested code and its absmax
    code2_t = torch.linspace(-1, 1, 256, device=dev, dtype=torch.float32)
    bnb_a2 = torch.rand((nb + 255) // 256, device=dev) * 0.01 + 1e-3
    # mixs: absmax bytes then 1024 nested absmax floats in one buffer
    scal = torch.cat([a1_0.view(torch.uint8), a2_0[:1024].view(torch.uint8)]) if nb % 4 == 0 else None
    torch.cuda.synchronize()

    def maker(spec):
        parts = spec.split(":")
        if parts[0] == "bnb" or parts[0].endswith("@bnb"):
            L = libs["prod" if parts[0] == "bnb" else parts[0][:-4]]

            def f(i):
                q, a1, _ = ins[i % PI]
                rc = L.nf4_dequant_bnb(q.data_ptr(), a1.data_ptr(), nb, code2_t.data_ptr(), bnb_a2.data_ptr(),
                                       bnb_a2.numel(), ctypes.c_float(BNB_OFFSET), outs[i % PO].data_ptr(),
                                       _lib.BF16, m * n, 64, 256, sp)
                if rc:
                    raise RuntimeError(_lib.strerror(rc))
            return f
        name16 = parts[0][:-3] if parts[0].endswith("@16") else None
        if parts[0] in ("prod", "prod16") or parts[0] in libs or name16 in libs:
            L = libs["prod" if parts[0] == "prod16" else (name16 or parts[0])]
            code = _lib.F16 if (parts[0] == "prod16" or name16) else _lib.BF16

            def f(i):
                q, a1, a2 = ins[i % PI]
                rc = L.nf4_dequant_ref(q.data_ptr(), nbytes, a1.data_ptr(), nb, a2.data_ptr(), n2,
                                       outs[i % PO].data_ptr(), code, m, n, sp)
                if rc:
                    raise RuntimeError(_lib.strerror(rc))
            return f
        kind = KIND[parts[0]]
        v = [int(x) for x in parts[1:]]
        if parts[0] == "mix":
            ld, stp, tpw = v
        elif parts[0] == "rd":
            ld, stp, tpw = v[0], 0, v[1]
        elif parts[0] == "wr":
            ld, stp, tpw = 0, v[0], v[1]
        elif parts[0] == "emptydiv":
            ld, stp, tpw = 0, 0, v[0]
        elif parts[0] == "mixs":
            ld, stp, tpw = 2, v[0], v[1]
        else:
            ld, stp, tpw = 0, 0, 1

        def f(i):
            rc = P.twin_launch(kind, ld, stp, tpw, ins[i % PI][0].data_ptr(), nbytes, outs[i % PO].data_ptr(),
                               (scal if kind == 6 else sink).data_ptr(), sp)
            if rc:
                raise RuntimeError(f"twin_launch {spec}: {rc}")
        return f

    specs = [s for s in args.kernels.split(",") if s]
    fns = {s: maker(s) for s in specs}
    steps = [int(v) for v in args.steps.split(",")]

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    torch.cuda._sleep(2_000_000)
    e1.record(st)
    torch.cuda.synchronize()
    cyc_per_us = 2_000_000 / max(e0.elapsed_time(e1) * 1e3, 1.0)
    for f in fns.values():  # every set touched once (TLB-warm)
        for i in range(max(PI, PO)):
            f(i)
    torch.cuda.synchronize()
    res = {(s, k): [] for s in specs for k in steps}
    for _ in range(args.rounds):
        for s in specs:
            f = fns[s]
            for k in steps:
                for i in range(max(PI, PO)):
                    f(i)
                if args.idle_ms:
                    torch.cuda.synchronize()
                    time.sleep(args.idle_ms * 1e-3)
                torch.cuda._sleep(int(cyc_per_us * (30.0 * (k + args.lead) + 200.0)))
                for j in range(args.lead):
                    f(j - args.lead + 10 * PI * PO)
                e0.record(st)
                for i in range(k):
                    f(i)
                e1.record(st)
                torch.cuda.synchronize()
                res[(s, k)].append(e0.elapsed_time(e1) * 1e3 / k)
    # hygiene: every dequant library's output of set 0 vs the C oracle (first 32 rows)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np

    import nf4_oracle as Ora

    checked = {}
    for s in specs:
        if s == "bnb" or s.endswith("@bnb"):
            outs[0].zero_()
            fns[s](0)
            torch.cuda.synchronize()
            r = 32
            want = Ora.COracle().dequant_bnb(p0[: r * n // 2], a10, code2_t.cpu().numpy(), bnb_a2.cpu().numpy(),
                                             np.float32(BNB_OFFSET), r * n, Ora.BF16, 64, 256)
            got = outs[0][:r].contiguous().view(torch.int16).cpu().numpy().view(np.uint16).reshape(-1)
            checked[s] = bool(np.array_equal(got, want.reshape(-1)))
            continue
        if s.split(":")[0] in ("prod", "prod16") or s in libs or s[:-3] in libs:
            outs[0].zero_()
            fns[s](0)
            torch.cuda.synchronize()
            r = 32
            code = Ora.F16 if (s == "prod16" or s.endswith("@16")) else Ora.BF16
            want = Ora.dequant_ref_np(p0[: r * n // 2], a10, a20, r, n, code)
            got = outs[0][:r].contiguous().view(torch.int16).cpu().numpy().view(np.uint16)
            checked[s] = bool(np.array_equal(got, want))
    for s in specs:
        for k in steps:
            ts = sorted(res[(s, k)])
            med = ts[len(ts) // 2]
            print(json.dumps({"tag": args.tag, "kernel": s, "m": m, "n": n, "steps": k, "rounds": args.rounds,
                              "in_sets": PI, "out_sets": PO, "idle_ms": args.idle_ms, "checked": checked.get(s),
                              "us_median": round(med, 3), "us_min": round(ts[0], 3), "us_max": round(ts[-1], 3),
                              "dequant_frac_at_this_time": round(alg / (med * 1e-6) / PEAK, 4)}), flush=True)


if __name__ == "__main__":
    main()
