"""Generate tests/golden/ by running the REFERENCE fallback on deterministic inputs.

Run here (in the build container, where /root/reference exists):

    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden.py

It imports ``_aggressive_pytorch_t4``
(/root/reference/nf4_triton_dequantization/kernel_optimized.py:208-314), the
reference's pure-PyTorch path, calls it on duck-typed modules built from the
splitmix64 inputs of ``oracle/nf4_oracle.py``, and writes

* ``tests/golden/<case>.npz``  -- inputs + expected output bits (small cases);
* ``tests/golden/manifest.json`` -- per case: shape, dtype, seeds, sha256 of the
  output bytes, and for big cases ~4K sampled (flat index, bits) pairs.

With ``--triton-interp`` it also runs the reference Triton path
(``_triton_dequantize_main``, :142-205) under ``TRITON_INTERPRET=1`` on the
small fp16 cases and records whether it agrees with the fallback bit for bit
(the interpreter truncates bf16, SURVEY §0.1, so bf16 is not compared).

Nothing under /root/reference is copied: only the generated data is committed.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys
from types import SimpleNamespace

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import nf4_oracle as O  # noqa: E402

REF = "/root/reference"
GOLDEN = os.path.join(REPO, "tests", "golden")

# (name, m, n, dtype, seed, overrides)
SMALL_CASES = [
    ("c16x128_f16", 16, 128, "f16", 11, {}),
    ("c64x512_bf16", 64, 512, "bf16", 12, {}),
    ("c8x96_f16_partial_nbwrap", 8, 96, "f16", 13, {"nb": 5}),
    ("c3x128_bf16_n2trunc", 3, 128, "bf16", 14, {"n2": 17}),
    ("c2x11008_bf16_g43", 2, 11008, "bf16", 15, {}),
    ("c32x256_bf16_neg_a2", 32, 256, "bf16", 16, {"a2_kind": "normal"}),
    ("c32x256_f16_neg_a2", 32, 256, "f16", 17, {"a2_kind": "normal"}),
    ("c5x77_f16_odd_n", 5, 77, "f16", 18, {"stride": 39}),
    ("c1x64_bf16_min", 1, 64, "bf16", 19, {}),
    ("c7x192_bf16_bpr3", 7, 192, "bf16", 20, {}),
    ("c4x320_f16_tiny_nb_n2", 4, 320, "f16", 21, {"nb": 3, "n2": 1}),
    ("c16x256_f16_overflow", 16, 256, "f16", 22, {"a2_scale": 4.0e5}),
    ("c16x256_f16_subnormal", 16, 256, "f16", 23, {"a2_scale": 1.0e-5}),
    ("c16x256_bf16_denorm_a2", 16, 256, "bf16", 24, {"a2_scale": 1.0e-37}),
    ("c24x1024_bf16_a2_fp16", 24, 1024, "bf16", 25, {"a2_dtype": "f16"}),
    ("c9x136_bf16_rowpad", 9, 136, "bf16", 26, {"stride": 72}),
    ("c12x256_f16_single", 12, 256, "f16", 27, {"single": 0}),
    ("c6x200_bf16_single_wide", 6, 200, "bf16", 28, {"single": 3}),
]

BIG_CASES = [
    ("C1_1024x1024_f16", 1024, 1024, "f16", 3407, {}),
    ("C2_4096x4096_bf16", 4096, 4096, "bf16", 3409, {}),
    ("c64x11008_bf16", 64, 11008, "bf16", 3408, {}),
    ("c1024x4096_f16_neg", 1024, 4096, "f16", 3410, {"a2_kind": "normal"}),
    # BASELINE configs at full size (round 2): C4's fp16 leg, C5's per-GPU unit and
    # every distinct C3 shape (Llama-3-8B 1024/4096/14336 and Llama-2-7B 11008)
    ("C4_4096x4096_f16", 4096, 4096, "f16", 3409, {}),
    ("C5_8192x8192_bf16", 8192, 8192, "bf16", 3411, {}),
    ("C3_1024x4096_bf16", 1024, 4096, "bf16", 3420, {}),
    ("C3_14336x4096_bf16", 14336, 4096, "bf16", 3421, {}),
    ("C3_4096x14336_bf16", 4096, 14336, "bf16", 3422, {}),
    ("C3b_11008x4096_bf16", 11008, 4096, "bf16", 3423, {}),
    ("C3b_4096x11008_bf16", 4096, 11008, "bf16", 3424, {}),
]


def case_inputs(m, n, seed, ov):
    return O.golden_case_inputs(m, n, seed, ov)


def torch_module(packed, a1, a2, absmax_single, m, n, dtype, ov):
    import torch

    tdt = torch.float16 if dtype == "f16" else torch.bfloat16
    a2_t = torch.from_numpy(a2.copy())
    if ov.get("a2_dtype") == "f16":
        a2_t = a2_t.to(torch.float16)
    absmax = torch.from_numpy(absmax_single.copy()) if absmax_single is not None else torch.from_numpy(a1.copy())
    qs = SimpleNamespace(absmax=absmax, state2=SimpleNamespace(absmax=a2_t), dtype=tdt)
    w = SimpleNamespace(data=torch.from_numpy(packed.copy()).view(-1, 1), quant_state=qs)
    return SimpleNamespace(weight=w, out_features=m, in_features=n)


def run_reference(mod):
    import torch

    sys.path.insert(0, REF)
    from nf4_triton_dequantization.kernel_optimized import _aggressive_pytorch_t4

    out = _aggressive_pytorch_t4(mod)
    return out.contiguous().view(torch.int16).numpy().view(np.uint16)


def sha(b: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(b).tobytes()).hexdigest()


def triton_interp_check(names):
    """Child process: TRITON_INTERPRET=1 reference Triton path vs fallback (fp16)."""
    code = r"""
import json, sys, os
sys.path.insert(0, %r); sys.path.insert(0, %r)
import numpy as np, torch
import gen_golden as G
from nf4_triton_dequantization.kernel_optimized import _triton_dequantize_main
res = {}
for name, m, n, dt, seed, ov in G.SMALL_CASES:
    if name not in %r: continue
    p, a1, a2, s = G.case_inputs(m, n, seed, ov)
    mod = G.torch_module(p, a1, a2, s, m, n, dt, ov)
    mod.weight.data = mod.weight.data.view(-1)
    try:
        out = _triton_dequantize_main(mod).contiguous().view(torch.int16).numpy().view(np.uint16)
        res[name] = G.sha(out)
    except Exception as e:
        res[name] = 'error: %%s' %% type(e).__name__
print('JSON' + json.dumps(res))
""" % (HERE, REF, list(names))
    env = dict(os.environ, TRITON_INTERPRET="1", PYTHONDONTWRITEBYTECODE="1")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=1800)
    for line in p.stdout.splitlines():
        if line.startswith("JSON"):
            return json.loads(line[4:])
    raise RuntimeError("triton interpreter check failed:\n" + p.stderr[-2000:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--triton-interp", action="store_true")
    ap.add_argument("--only", default="", help="comma-separated case names: (re)generate just these and keep "
                                               "every other entry of the existing manifest")
    args = ap.parse_args()
    os.makedirs(GOLDEN, exist_ok=True)
    only = {x for x in args.only.split(",") if x}
    manifest = {"generator": "oracle/gen_golden.py",
                "reference": "nf4_triton_dequantization/kernel_optimized.py:208-314 (_aggressive_pytorch_t4)",
                "cases": {}}
    samples = {}
    if only:
        with open(os.path.join(GOLDEN, "manifest.json")) as f:
            manifest = json.load(f)
        with np.load(os.path.join(GOLDEN, "big_samples.npz"), allow_pickle=False) as z:
            samples = {k: z[k] for k in z.files}
    for big, cases in ((False, SMALL_CASES), (True, BIG_CASES)):
        for name, m, n, dt, seed, ov in cases:
            if only and name not in only:
                continue
            packed, a1, a2, single = case_inputs(m, n, seed, ov)
            mod = torch_module(packed, a1, a2, single, m, n, dt, ov)
            out = run_reference(mod)
            entry = {"m": m, "n": n, "dtype": dt, "seed": seed, "overrides": ov,
                     "sha256": sha(out), "nan_count": int(np.isnan(out.view(np.float16) if dt == "f16" else
                                                                   (out.astype(np.uint32) << 16).view(np.float32)).sum())}
            if big:
                rng = np.random.default_rng(seed)
                idx = np.sort(rng.choice(out.size, size=min(4096, out.size), replace=False))
                samples[name + "/idx"] = idx.astype(np.int64)
                samples[name + "/bits"] = out.reshape(-1)[idx]
                entry["samples"] = "big_samples.npz"
            else:
                arrays = {"packed": packed, "a1": a1, "a2": a2, "out_bits": out}
                if ov.get("a2_dtype") == "f16":     # what the path sees after .to(float32) (:182)
                    arrays["a2_f16"] = a2.astype(np.float16)
                    arrays["a2"] = arrays["a2_f16"].astype(np.float32)
                if single is not None:
                    arrays["absmax_f32"] = single
                np.savez_compressed(os.path.join(GOLDEN, name + ".npz"), **arrays)
                entry["file"] = name + ".npz"
            manifest["cases"][name] = entry
            print(f"{name:34s} {m}x{n} {dt} sha={entry['sha256'][:16]}")
    if args.triton_interp:
        names = [c[0] for c in SMALL_CASES if c[3] == "f16" and "single" not in c[5]]
        got = triton_interp_check(names)
        manifest["triton_interpret_fp16"] = {
            k: {"sha256": v, "agrees_with_fallback": v == manifest["cases"][k]["sha256"]} for k, v in got.items()}
        for k, v in manifest["triton_interpret_fp16"].items():
            print(f"triton-interp {k:30s} agrees={v['agrees_with_fallback']}")
    np.savez_compressed(os.path.join(GOLDEN, "big_samples.npz"), **samples)
    with open(os.path.join(GOLDEN, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
