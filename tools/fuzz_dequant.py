"""Randomised parity sweep of the drop-in dequant against the C oracle (tools only).

    python tools/fuzz_dequant.py [--cases 2000] [--seed 1] [--seconds 600] > fuzz.jsonl

Each case draws a shape (1-300 rows, 1-4100 columns: odd widths, partial 64-blocks,
whole-tile multiples), an output dtype (fp16 / bf16 / fp32), a packed row stride (n/2
or padded), the absmax sizes (the reference's full counts, or short ones that exercise
its repeat-wrap) and the sign of the nested absmax. It runs
``triton_dequantize_nf4`` on the GPU (flat or chunk kernel, as the library picks) and
compares every output bit with the C oracle (``nf4o_dequant_ref``), which is pinned to
the reference fallback (tests/golden/). With ``--abi-rate p`` a fraction p of the cases
calls the C ABI (``nf4_dequant_ref``) instead, with the packed weight 0-3 bytes and the
output 0-7 elements into their allocations and a sentinel on both sides of the output
(every load / store form of the chunk kernel, and no write outside the output).
Mismatching cases are printed with their parameters. One progress line per 200 cases,
then a summary line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import nf4_oracle as O  # noqa: E402  -- the checker
from _helpers import make_module, out_bits  # noqa: E402
from nf4_triton_dequantization_amd import triton_dequantize_nf4  # noqa: E402

DT = {"f16": O.F16, "bf16": O.BF16, "f32": O.F32}


def draw(rng):
    m = int(rng.integers(1, 301))
    kind = rng.integers(0, 4)
    if kind == 0:
        n = int(rng.integers(1, 130))                   # tiny, odd widths
        if rng.random() < 0.3:
            m = int(rng.integers(300, 3001))            # many rows per wave
    elif kind == 1:
        n = 64 * int(rng.integers(1, 65))               # whole 64-blocks (flat kernel)
    elif kind == 2:
        n = 2 * int(rng.integers(1, 2051))              # even widths, partial blocks
    else:
        n = int(rng.integers(1, 4101))
    dt = ["f16", "bf16", "f32"][int(rng.integers(0, 3))]
    ov = {"stride": (n + 1) // 2 + (int(rng.integers(1, 9)) if rng.random() < 0.15 else 0)}
    nb_full = (m * n + 63) // 64
    if rng.random() < 0.25:
        ov["nb"] = int(rng.integers(1, nb_full + 1))     # short absmax: the reference's repeat-wrap
    nb = ov.get("nb", nb_full)
    if rng.random() < 0.25:
        ov["n2"] = int(rng.integers(1, (nb + 255) // 256 + 2))
    if rng.random() < 0.5:
        ov["a2_kind"] = "normal"
    return m, n, dt, ov


def abi_case(dev, p, a1, a2, m, n, dt, poff, ooff, want, guard=64):
    """nf4_dequant_ref with the packed weight `poff` bytes and the output `ooff` elements
    into their allocations; True if the output matches and the guards are untouched."""
    from nf4_triton_dequantization_amd import _lib

    tdt = {"f16": torch.float16, "bf16": torch.bfloat16, "f32": torch.float32}[dt]
    ibits = torch.int32 if dt == "f32" else torch.int16
    sentinel = 0x5A5A5A5A if dt == "f32" else 0x5A5A
    big = torch.zeros(p.size + 8, dtype=torch.uint8, device=dev)
    big[poff:poff + p.size] = torch.from_numpy(p).to(dev)
    t1, t2 = torch.from_numpy(a1).to(dev), torch.from_numpy(a2).to(dev)
    buf = torch.empty(guard + ooff + m * n + (1 << 18), dtype=tdt, device=dev)  # (wide after: stray spans)
    buf.view(ibits).fill_(sentinel)
    start = guard + ooff
    rc = _lib.lib().nf4_dequant_ref(big.data_ptr() + poff, p.size, t1.data_ptr(), t1.numel(), t2.data_ptr(),
                                    t2.numel(), buf.data_ptr() + start * buf.element_size(), DT[dt], m, n,
                                    torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        return False
    bits = buf.view(ibits).cpu().numpy()
    if not ((bits[:start] == sentinel).all() and (bits[start + m * n:] == sentinel).all()):
        return False
    got = bits[start:start + m * n].view(np.uint32 if dt == "f32" else np.uint16).reshape(want.shape)
    return bool(np.array_equal(got, want))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=600.0)
    ap.add_argument("--abi-rate", type=float, default=0.0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    orc = O.COracle()
    rng = np.random.default_rng(args.seed)
    t0 = time.time()
    done = bad = elements = 0
    kinds = {"f16": 0, "bf16": 0, "f32": 0}
    for i in range(args.cases):
        if time.time() - t0 > args.seconds:
            break
        m, n, dt, ov = draw(rng)
        seed = int(rng.integers(1, 1 << 30))
        p, a1, a2, _ = O.golden_case_inputs(m, n, seed, ov)
        want = orc.dequant_ref(p, a1, a2, m, n, DT[dt])
        if rng.random() < args.abi_rate:
            poff, ooff = int(rng.integers(0, 4)), int(rng.integers(0, 64))
            ov = dict(ov, packed_offset=poff, out_offset=ooff)
            ok = abi_case(dev, p, a1, a2, m, n, dt, poff, ooff, want)
        else:
            got = out_bits(triton_dequantize_nf4(make_module(p, a1, a2, m, n, dt, dev)))
            ok = np.array_equal(got.reshape(want.shape), want)
        done += 1
        elements += m * n
        kinds[dt] += 1
        if not ok:
            bad += 1
            print(json.dumps({"mismatch": {"m": m, "n": n, "dtype": dt, "seed": seed, "ov": ov}}), flush=True)
        if done % 200 == 0:
            print(json.dumps({"progress": done, "mismatches": bad, "seconds": round(time.time() - t0, 1)}), flush=True)
    print(json.dumps({"summary": {"cases": done, "mismatches": bad, "elements": elements, "by_dtype": kinds,
                                  "seed": args.seed, "seconds": round(time.time() - t0, 1)}}), flush=True)


if __name__ == "__main__":
    main()
