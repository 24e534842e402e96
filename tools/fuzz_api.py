"""Randomised parity sweep of the multi-weight and single-quant entry points (tools only).

    python tools/fuzz_api.py [--rounds 400] [--seed 1] [--seconds 500] > fuzz_api.jsonl

Each round draws one of three cases:
  many     ``dequantize_nf4_many`` over 1-40 weights of mixed shapes, dtypes, padded
           strides and short (wrapping) absmax. Batched launches are split by
           NF4DQ_BATCH_MAX; every output is compared bit for bit with the C oracle.
  single   the reference's single-quant branch (fp32 absmax, ``triton_dequantize_nf4`` ->
           ``nf4_dequant_single``), bit for bit against ``nf4o_dequant_single``.
  grouped  ``nf4_linear_grouped`` over 2-8 weights that share x (random N each, one K,
           M <= 32), each output against the float64 oracle product with the GEMM suite's
           tolerance.
One progress line per 50 rounds, then a summary.
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
from nf4_triton_dequantization_amd import dequantize_nf4_many, nf4_linear_grouped, triton_dequantize_nf4  # noqa: E402

DT = {"f16": O.F16, "bf16": O.BF16, "f32": O.F32}


def shape(rng):
    m = int(rng.integers(1, 200))
    n = 64 * int(rng.integers(1, 40)) if rng.random() < 0.6 else int(rng.integers(1, 1500))
    return m, n


def overrides(rng, m, n):
    ov = {"stride": (n + 1) // 2 + (int(rng.integers(1, 5)) if rng.random() < 0.1 else 0)}
    if rng.random() < 0.2:
        ov["nb"] = int(rng.integers(1, (m * n + 63) // 64 + 1))
    if rng.random() < 0.5:
        ov["a2_kind"] = "normal"
    return ov


def bits_to_f64(bits, dt):
    if dt == "f16":
        return bits.view(np.float16).astype(np.float64)
    return (bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=400)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=500.0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    orc = O.COracle()
    rng = np.random.default_rng(args.seed)
    t0 = time.time()
    counts = {"many": 0, "many_weights": 0, "single": 0, "grouped": 0, "grouped_weights": 0}
    bad = 0
    for r in range(args.rounds):
        if time.time() - t0 > args.seconds:
            break
        kind = ["many", "single", "grouped"][int(rng.integers(0, 3))]
        seed = int(rng.integers(1, 1 << 30))
        if kind == "many":
            mods, wants, dts = [], [], []
            for j in range(int(rng.integers(1, 41))):
                m, n = shape(rng)
                dt = ["f16", "bf16", "f32"][int(rng.integers(0, 3))]
                p, a1, a2, _ = O.golden_case_inputs(m, n, seed + j, overrides(rng, m, n))
                wants.append(orc.dequant_ref(p, a1, a2, m, n, DT[dt]))
                mods.append(make_module(p, a1, a2, m, n, dt, dev))
                dts.append(dt)
            outs = dequantize_nf4_many(mods)
            for j, (o, w) in enumerate(zip(outs, wants)):
                if not np.array_equal(out_bits(o).reshape(w.shape), w):
                    bad += 1
                    print(json.dumps({"mismatch": {"kind": kind, "seed": seed, "index": j, "shape": list(w.shape),
                                                   "dtype": dts[j]}}), flush=True)
            counts["many"] += 1
            counts["many_weights"] += len(mods)
        elif kind == "single":
            m, n = shape(rng)
            dt = ["f16", "bf16", "f32"][int(rng.integers(0, 3))]
            p, a1, a2, single = O.golden_case_inputs(m, n, seed, {"single": int(rng.integers(0, 3)),
                                                                  "stride": (n + 1) // 2})
            want = orc.dequant_single(p, single, m, n, DT[dt])
            got = out_bits(triton_dequantize_nf4(make_module(p, single, a2, m, n, dt, dev)))
            if not np.array_equal(got.reshape(want.shape), want):
                bad += 1
                print(json.dumps({"mismatch": {"kind": kind, "seed": seed, "m": m, "n": n, "dtype": dt}}), flush=True)
            counts["single"] += 1
        else:
            M = int(rng.integers(1, 33))
            K = 128 * int(rng.integers(1, 33))
            dt = "bf16" if rng.random() < 0.6 else "f16"
            g = int(rng.integers(2, 9))
            Ns = [64 * int(rng.integers(1, 33)) for _ in range(g)]
            x = O.normal_f32(seed, M * K, stream=9).reshape(M, K)
            xt = torch.from_numpy(x).to(torch.bfloat16 if dt == "bf16" else torch.float16)
            xf = bits_to_f64(xt.view(torch.int16).numpy().view(np.uint16), dt)
            mods, wfs = [], []
            for j, N in enumerate(Ns):
                ov = {"a2_kind": "normal"} if rng.random() < 0.5 else {}
                p, a1, a2, _ = O.golden_case_inputs(N, K, seed + 17 * j, ov)
                wfs.append(bits_to_f64(orc.dequant_ref(p, a1, a2, N, K, DT[dt]), dt))
                mods.append(make_module(p, a1, a2, N, K, dt, dev))
            ys = nf4_linear_grouped(xt.to(dev), mods)
            p_, sub = (8, 2.0 ** -134) if dt == "bf16" else (10, 2.0 ** -25)
            for j, (y, wf) in enumerate(zip(ys, wfs)):
                ref = xf @ wf.T
                bound = 2.0 ** -p_ * np.abs(ref) + 2.0 ** -20 * (np.abs(xf) @ np.abs(wf).T) + sub
                got = bits_to_f64(y.contiguous().view(torch.int16).cpu().numpy().view(np.uint16), dt).reshape(ref.shape)
                if not (np.abs(got - ref) <= bound).all():
                    bad += 1
                    print(json.dumps({"mismatch": {"kind": kind, "seed": seed, "index": j, "M": M, "K": K, "Ns": Ns,
                                                   "dtype": dt}}), flush=True)
            counts["grouped"] += 1
            counts["grouped_weights"] += g
        if (r + 1) % 50 == 0:
            print(json.dumps({"progress": r + 1, "mismatches": bad, "seconds": round(time.time() - t0, 1)}), flush=True)
    print(json.dumps({"summary": {**counts, "mismatches": bad, "seed": args.seed,
                                  "seconds": round(time.time() - t0, 1)}}), flush=True)


if __name__ == "__main__":
    main()
