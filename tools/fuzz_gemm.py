"""Randomised parity sweep of the fused decode GEMM (tools only).

    python tools/fuzz_gemm.py [--cases 1500] [--seed 1] [--seconds 500] > fuzz_gemm.jsonl

Each case draws M (1-32), N (a multiple of 64 up to 3072), K (a multiple of 128 up to
6144), the dtype (bf16 / fp16), full or short absmax arrays (the reference's repeat-wrap)
and signed nested absmax. It then runs ``nf4_linear`` (the library's choice of kernel
and decomposition) and, for a share of the cases (``--cfg-rate``), an explicitly drawn
configuration of any of the six kernels through ``nf4_gemm_ref_cfg`` (invalid draws are
skipped; a split-K timeout flagged in the workspace counts as a failure). Each result is
checked against a float64 product of the C oracle's dequantized weights with the GEMM
suite's tolerance
(tests/test_gpu_gemm.py: 2^-p |ref| + 2^-20 sum|x w|). One progress line per 100
cases, then a summary.
"""
from __future__ import annotations

import argparse
import ctypes
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
from _helpers import make_module  # noqa: E402
from nf4_triton_dequantization_amd import _lib, nf4_linear  # noqa: E402


def bits_to_f64(bits, dt):
    if dt == "f16":
        return bits.view(np.float16).astype(np.float64)
    return (bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def tol(ref, mag, dt):
    p, sub = (8, 2.0 ** -134) if dt == "bf16" else (10, 2.0 ** -25)
    return 2.0 ** -p * np.abs(ref) + 2.0 ** -20 * mag + sub


def random_cfg(rng, M, N, K):
    """A drawn configuration of one of the six kernels (may be invalid: skipped)."""
    k = int(rng.choice([1, 2, 3, 4, 5, 7]))  # (6, the balanced kernel, was retired in round 6)
    if k == _lib.GEMM_GEMV:  # the decode GEMV: M = 1, K % 2048 == 0 (else rejected)
        return _lib.GemmCfg(k, int(rng.choice([8, 16])), int(rng.choice([1, 2, 4])), 1, int(rng.choice([0, 1, 2])))
    waves = int(rng.choice([4, 8, 16]))
    depth = int(rng.choice([1, 2, 4, 8]))
    strips = int(rng.choice([1, 2, 4]))
    if k == _lib.GEMM_XR:
        kpw = strips
        ks = -(-(K // 128) // (waves * kpw))
    elif k == _lib.GEMM_XS:
        ks = -(-(K // 128) // depth)
        strips = 1
    else:
        ks = int(rng.choice([1, 2, 4]))
    return _lib.GemmCfg(k, waves, depth, ks, strips)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=1500)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=500.0)
    ap.add_argument("--cfg-rate", type=float, default=0.25, help="share of cases that also run a drawn configuration")
    ap.add_argument("--gemv-rate", type=float, default=0.0,
                    help="share of cases at M = 1 with K % 2048 == 0 and N <= 4096 (the decode GEMV's domain)")
    ap.add_argument("--boundary-rate", type=float, default=0.1,
                    help="share of cases drawn from the default-rule boundary shapes (large N, K = 14336)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    orc = O.COracle()
    rng = np.random.default_rng(args.seed)
    t0 = time.time()
    done = bad = cfg_runs = 0
    for i in range(args.cases):
        if time.time() - t0 > args.seconds:
            break
        M = int(rng.integers(1, 33))
        N = 64 * int(rng.integers(1, 49))
        K = 128 * int(rng.integers(1, 49))
        if rng.random() < args.boundary_rate:
            # the default-rule boundaries the uniform draw cannot reach: M on
            # either side of 8 / 16 / 24, the wide launches (16-wave whole-K XR at
            # N >= 24576, persistent strips = 4 at N >= 8192) and the down projection's K
            M = int(rng.choice([1, 8, 9, 16, 17, 24, 25, 32]))
            N, K = [(1024, 4096), (4096, 4096), (8192, 4096), (14336, 4096), (24576, 4096), (28672, 4096),
                    (4096, 14336), (1024, 14336)][int(rng.integers(0, 8))]
        if rng.random() < args.gemv_rate:
            M, N, K = 1, 64 * int(rng.integers(1, 65)), 2048 * int(rng.integers(1, 9))
        dt = "bf16" if rng.random() < 0.6 else "f16"
        nb_full = N * K // 64
        ov = {"a2_kind": "normal" if rng.random() < 0.5 else "uniform"}
        if rng.random() < 0.2:
            ov["nb"] = int(rng.integers(1, nb_full + 1))
        seed = int(rng.integers(1, 1 << 30))
        p, a1, a2, _ = O.golden_case_inputs(N, K, seed, ov)
        w = orc.dequant_ref(p, a1, a2, N, K, O.BF16 if dt == "bf16" else O.F16)
        x = O.normal_f32(seed + 1, M * K, stream=9).reshape(M, K)
        xt = torch.from_numpy(x).to(torch.bfloat16 if dt == "bf16" else torch.float16)
        xb = xt.view(torch.int16).numpy().view(np.uint16)
        xf, wf = bits_to_f64(xb, dt), bits_to_f64(w, dt)
        ref = xf @ wf.T
        bound = tol(ref, np.abs(xf) @ np.abs(wf).T, dt)
        mod = make_module(p, a1, a2, N, K, dt, dev)
        outs = [("default", nf4_linear(xt.to(dev), mod))]
        if rng.random() < args.cfg_rate:
            cfg = random_cfg(rng, M, N, K)
            wsz = L.nf4_gemm_workspace_bytes_cfg(M, N, K, ctypes.byref(cfg))
            ws = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=dev)
            y = torch.empty((M, N), dtype=xt.dtype, device=dev)
            q = mod.weight.data
            qs = mod.weight.quant_state
            rc = L.nf4_gemm_ref_cfg(xt.to(dev).data_ptr(), M, q.data_ptr(), q.numel(), qs.absmax.data_ptr(),
                                    qs.absmax.numel(), qs.state2.absmax.data_ptr(), qs.state2.absmax.numel(),
                                    y.data_ptr(), _lib.BF16 if dt == "bf16" else _lib.F16, N, K,
                                    ws.data_ptr() if wsz else None, wsz, ctypes.byref(cfg),
                                    torch.cuda.current_stream().cuda_stream)
            if rc == 0:
                cfg_runs += 1
                label = [cfg.kernel, cfg.waves, cfg.depth, cfg.ksplit, cfg.strips]
                if wsz and L.nf4_gemm_check_workspace(ws.data_ptr(), wsz, torch.cuda.current_stream().cuda_stream):
                    bad += 1
                    print(json.dumps({"timeout": {"M": M, "N": N, "K": K, "cfg": label, "seed": seed}}), flush=True)
                outs.append((label, y))
        for label, y in outs:
            got = bits_to_f64(y.contiguous().view(torch.int16).cpu().numpy().view(np.uint16), dt).reshape(M, N)
            if not (np.abs(got - ref) <= bound).all():
                bad += 1
                print(json.dumps({"mismatch": {"M": M, "N": N, "K": K, "dtype": dt, "seed": seed, "ov": ov,
                                               "path": label,
                                               "worst": float(np.abs(got - ref).max())}}), flush=True)
        done += 1
        if done % 100 == 0:
            print(json.dumps({"progress": done, "mismatches": bad, "cfg_runs": cfg_runs,
                              "seconds": round(time.time() - t0, 1)}), flush=True)
    print(json.dumps({"summary": {"cases": done, "explicit_cfg_runs": cfg_runs, "mismatches": bad,
                                  "seed": args.seed, "seconds": round(time.time() - t0, 1)}}), flush=True)


if __name__ == "__main__":
    main()
