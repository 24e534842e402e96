"""The chunk kernel against the flat kernel, HBM-streamed, interleaved rounds (tools only).

    python tools/chunk_ab.py [--rounds 7] [--steps 64]

Cases (bf16, bench.py's rotation: >= 512 MiB of distinct reads and of writes; eager
launches behind a spin, as bench.py times its steps):
  flat_4096     4096x4096 through the default path (the flat kernel)
  chunk_4096    the same matrices through the chunk kernel (nf4_dequant_ref_cfg flags =
                NF4DQ_CFG_CHUNKS): the kernel's own cost on the flat kernel's stream
  chunk_4080    4096x4080 (n % 64 != 0): the chunk kernel, as the drop-in runs it
  rows_4080     4096x4080 through the one-thread-per-byte kernel (NF4DQ_CFG_ROWS)
  chunk_4095    4096x4095 (odd n: 2-byte stores)
  chunk_4090    4096x4090 (n % 8 == 2: 4-byte stores)
  pad_4096      4096x4096 with packed rows of 2052 bytes (the general form, dword loads)
  unal_4096     4096x4096 with the packed weight at an odd address (the piece kernel since round 6)
  oal_4096      4096x4096 with the output one element off 16-byte alignment
  chunk_4100    4096x4100 (a row's last block holds 4 elements)
  padodd_4090   4096x4090 with packed rows of 2048 bytes (padded, n % 8 != 0)
--dtype f32 / f16: the output type (default bf16).
--libs a,b: the same cases through other builds of the library (tools/_build/libnf4dq_<x>.so),
interleaved, tagged "<x>:<case>".
Prints one JSON line per case: median / min / max us per launch and the fraction of
8 TB/s (SURVEY §8d algorithmic bytes).
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
sys.path.insert(0, os.path.join(REPO, "tools"))
from nf4_triton_dequantization_amd import _lib  # noqa: E402
from bench_configs import PEAK, alg_bytes, rotating_sets, rotation  # noqa: E402

SHAPES = {"flat_4096": (4096, 4096, 0), "chunk_4096": (4096, 4096, _lib.CFG_CHUNKS),
          "chunk_4080": (4096, 4080, 0), "rows_4080": (4096, 4080, _lib.CFG_ROWS),
          "chunk_4095": (4096, 4095, 0), "chunk_4090": (4096, 4090, 0),
          "pad_4096": (4096, 4096, 0), "unal_4096": (4096, 4096, 0), "oal_4096": (4096, 4096, 0),
          "chunk_4100": (4096, 4100, 0), "padodd_4090": (4096, 4090, 0)}
# pad_4096: packed rows of 2052 bytes (n % 64 == 0 but not dense: the general form with
# dword loads); unal_4096: the packed weight one byte into its allocation (alignbyte loads)
PAD = {"pad_4096": 4, "padodd_4090": 3}
UNAL = {"unal_4096": 1}
OOFF = {"oal_4096": 1}  # output element offset


def case_key(name):
    m, n, _ = SHAPES[name]
    return (m, n, PAD.get(name, 0), UNAL.get(name, 0), OOFF.get(name, 0))


TDT = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}
DT = TDT["bf16"]  # (set by --dtype)


def case_sets(name, dev, gen):
    """(input sets, output sets) of a case, rotated as bench.py rotates (>= 512 MiB of
    distinct reads and of writes: HBM-streamed)."""
    m, n, _ = SHAPES[name]
    key = case_key(name)
    pin, pout = rotation(m, n, DT.itemsize)
    if n % 2 or key[2] or key[3] or key[4]:  # packed rows of ceil(n/2) + pad bytes, at byte offset unal
        ins = []
        stride = (n + 1) // 2 + key[2]
        for _ in range(pin):
            nb = m * n // 64 + 1
            q = torch.randint(0, 256, (m * stride + key[3],), dtype=torch.uint8, device=dev, generator=gen)
            ins.append((q[key[3]:],
                        torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=gen),
                        torch.rand((nb + 255) // 256, device=dev, generator=gen) * 0.01 + 1e-3))
        outs = [torch.empty((m * n + 64,), dtype=DT, device=dev)[key[4]:] for _ in range(pout)]
        return ins, outs
    return rotating_sets(m, n, DT, dev, gen, pin, pout)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--cases", default="flat_4096,chunk_4096,chunk_4080,rows_4080,chunk_4095,chunk_4090")
    ap.add_argument("--libs", default="")
    ap.add_argument("--dtype", default="bf16", choices=sorted(TDT))
    args = ap.parse_args()
    global DT
    DT = TDT[args.dtype]
    dcode = {"bf16": _lib.BF16, "f16": _lib.F16, "f32": _lib.F32}[args.dtype]
    dev = torch.device("cuda", 0)
    libs = {"prod": _lib.lib()}
    for path in [v for v in args.libs.split(",") if v]:
        h = ctypes.CDLL(os.path.abspath(path))
        for fname, (res_t, argt) in _lib.SIGNATURES.items():
            fn = getattr(h, fname, None)
            if fn is not None:
                fn.restype, fn.argtypes = res_t, argt
        libs[os.path.basename(path).replace("libnf4dq_", "").replace(".so", "")] = h
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    torch.cuda._sleep(2_000_000)
    e1.record(st)
    torch.cuda.synchronize()
    cyc_per_us = 2_000_000 / max(e0.elapsed_time(e1) * 1e3, 1.0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    sets = {}
    for name in args.cases.split(","):
        key = case_key(name)
        if key not in sets:
            sets[key] = case_sets(name, dev, gen)
    cfgs = {f: _lib.LaunchCfg(4, 0, 1, f) for f in (_lib.CFG_CHUNKS, _lib.CFG_ROWS)}

    def launcher(tag):
        lname, name = tag.split(":")
        L = libs[lname]
        m, n, flags = SHAPES[name]
        ins, outs = sets[case_key(name)]

        def launch(i):
            q, a1, a2 = ins[i % len(ins)]
            o = outs[i % len(outs)]
            if flags:
                rc = L.nf4_dequant_ref_cfg(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(),
                                           a2.numel(), o.data_ptr(), dcode, m, n, ctypes.byref(cfgs[flags]),
                                           st.cuda_stream)
            else:
                rc = L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                       o.data_ptr(), dcode, m, n, st.cuda_stream)
            assert rc == 0, rc
        return launch

    names = [f"{lib}:{c}" for c in args.cases.split(",") for lib in libs]
    fns = {nm: launcher(nm) for nm in names}
    for nm in names:  # every set touched once
        c = nm.split(":")[1]
        ins, outs = sets[case_key(c)]
        for i in range(max(len(ins), len(outs))):
            fns[nm](i)
    torch.cuda.synchronize()
    res = {nm: [] for nm in names}
    for _ in range(args.rounds):
        for nm in names:
            torch.cuda._sleep(int(cyc_per_us * (40.0 * (args.steps + 8) + 200.0)))
            for j in range(8):
                fns[nm](j - 8)
            e0.record(st)
            for i in range(args.steps):
                fns[nm](i)
            e1.record(st)
            torch.cuda.synchronize()
            res[nm].append(e0.elapsed_time(e1) * 1e3 / args.steps)
    for nm in names:
        m, n, flags = SHAPES[nm.split(":")[1]]
        ts = sorted(res[nm])
        med = ts[len(ts) // 2]
        byt = alg_bytes(m, n, DT.itemsize)
        print(json.dumps({"case": nm, "m": m, "n": n, "dtype": args.dtype, "flags": flags, "steps": args.steps, "rounds": args.rounds,
                          "us_median": round(med, 3), "us_min": round(ts[0], 3), "us_max": round(ts[-1], 3),
                          "frac": round(byt / (med * 1e-6) / PEAK, 4)}), flush=True)


if __name__ == "__main__":
    main()
