"""Randomised parity sweep of the drop-in dequant against the C oracle (tools only).

    python tools/fuzz_dequant.py [--cases 2000] [--seed 1] [--seconds 600] > fuzz.jsonl

Each case draws a shape (1-300 rows, 1-4100 columns: odd widths, partial 64-blocks,
whole-tile multiples), an output dtype (fp16 / bf16 / fp32), a packed row stride (n/2
or padded), the absmax sizes (the reference's full counts, or short ones that exercise
its repeat-wrap) and the sign of the nested absmax. It runs
``triton_dequantize_nf4`` on the GPU (flat or rows kernel, as the library picks) and
compares every output bit with the C oracle (``nf4o_dequant_ref``), which is pinned to
the reference fallback (tests/golden/). Mismatching cases are printed with their
parameters. One progress line per 200 cases, then a summary line.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=600.0)
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
