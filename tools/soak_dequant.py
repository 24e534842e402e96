"""Soak of the dequant kernels (tools only): every kernel form launched for a long time,
outputs checked bit for bit against the C oracle throughout.

    python tools/soak_dequant.py [--seconds 600] [--check-every 64]

Forms (fixed inputs per form, expected outputs computed once by the C oracle):
  flat_bf16 / flat_f16 / flat_f32   4096x4096 (the flat kernel)
  dense_bf16                        4096x4080 (the chunk kernel's dense form)
  padded_bf16                       1024x4096 with packed rows of 2052 bytes (general form)
  odd_f16                           777x4095 (n % 8 != 0: the LDS-staged stores)
  unaligned_bf16                    513x1000, packed weight at an odd address (byte loads)
  single_bf16                       1000x4080 single-quant (fp32 absmax)
  batched_bf16                      Llama-3-8B layer (7 weights) through nf4_dequant_ref_batched
Each iteration launches every form into one of 4 rotating outputs per form; every
--check-every iterations the device synchronises and the most recent output of every
form is compared with its expected bits (and, for the misaligned outputs, the guard
elements around it).  A JSON progress line every ~30 s, then a summary.
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
import nf4_oracle as O  # noqa: E402  -- the checker
from nf4_triton_dequantization_amd import _lib  # noqa: E402

TDT = {O.F16: torch.float16, O.BF16: torch.bfloat16, O.F32: torch.float32}
IBITS = {O.F16: torch.int16, O.BF16: torch.int16, O.F32: torch.int32}
GUARD = 256


class Form:
    def __init__(self, name, m, n, dt, dev, orc, seed, pad=0, poff=0, ooff=0, single=False):
        self.name, self.m, self.n, self.dt, self.single = name, m, n, dt, single
        ov = {"stride": (n + 1) // 2 + pad}
        if single:
            ov["single"] = 1
        p, a1, a2, s1 = O.golden_case_inputs(m, n, seed, ov)
        self.want = (orc.dequant_single(p, s1, m, n, dt) if single else orc.dequant_ref(p, a1, a2, m, n, dt))
        self.want = self.want.view(np.int32 if dt == O.F32 else np.int16).reshape(-1)
        self.big = torch.zeros(p.size + 8, dtype=torch.uint8, device=dev)
        self.big[poff:poff + p.size] = torch.from_numpy(p).to(dev)
        self.pp, self.plen = self.big.data_ptr() + poff, p.size
        self.a1 = torch.from_numpy(a1).to(dev)
        self.a2 = torch.from_numpy(s1 if single else a2).to(dev)
        self.ooff = ooff
        self.outs = [torch.full((GUARD + ooff + m * n + GUARD,), 0, dtype=TDT[dt], device=dev) for _ in range(4)]
        self.last = 0

    def launch(self, L, i, st):
        o = self.outs[i % 4]
        self.last = i % 4
        optr = o.data_ptr() + (GUARD + self.ooff) * o.element_size()
        if self.single:
            rc = L.nf4_dequant_single(self.pp, self.plen, self.a2.data_ptr(), self.a2.numel(), optr, self.dt, self.m,
                                      self.n, st)
        else:
            rc = L.nf4_dequant_ref(self.pp, self.plen, self.a1.data_ptr(), self.a1.numel(), self.a2.data_ptr(),
                                   self.a2.numel(), optr, self.dt, self.m, self.n, st)
        assert rc == 0, (self.name, rc)

    def check(self):
        bits = self.outs[self.last].view(IBITS[self.dt]).cpu().numpy()
        s = GUARD + self.ooff
        ok = np.array_equal(bits[s:s + self.m * self.n], self.want)
        return ok and not bits[:s].any() and not bits[s + self.m * self.n:].any()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=600.0)
    ap.add_argument("--check-every", type=int, default=64)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    orc = O.COracle()
    orc.set_threads(16)
    L = _lib.lib()
    st = torch.cuda.current_stream().cuda_stream
    forms = [Form("flat_bf16", 4096, 4096, O.BF16, dev, orc, 11), Form("flat_f16", 4096, 4096, O.F16, dev, orc, 12),
             Form("flat_f32", 4096, 4096, O.F32, dev, orc, 13), Form("dense_bf16", 4096, 4080, O.BF16, dev, orc, 14),
             Form("padded_bf16", 1024, 4096, O.BF16, dev, orc, 15, pad=4),
             Form("odd_f16", 777, 4095, O.F16, dev, orc, 16, ooff=3),          # the piece kernel
             Form("piece_even_bf16", 1024, 4090, O.BF16, dev, orc, 19, poff=2, ooff=45),
             Form("padded_odd_f16", 777, 4095, O.F16, dev, orc, 20, pad=3, ooff=3),  # piece kernel, padded rows
             Form("staged_bf16", 3000, 510, O.BF16, dev, orc, 24, ooff=1),         # LDS-staged chunk form
             Form("piece32_f32", 1000, 4090, O.F32, dev, orc, 21, poff=1, ooff=3),  # fp32 piece kernel
             Form("tri_bf16", 1000, 4100, O.BF16, dev, orc, 22),                   # short last blocks
             Form("padded_f32", 512, 4096, O.F32, dev, orc, 23, pad=4),
             Form("unaligned_bf16", 513, 1000, O.BF16, dev, orc, 17, poff=1, ooff=1),
             Form("single_bf16", 1000, 4080, O.BF16, dev, orc, 18, single=True)]
    # one Llama-3-8B layer through the batched entry (flat pieces in one launch)
    shapes = [(4096, 4096), (1024, 4096), (1024, 4096), (4096, 4096), (14336, 4096), (14336, 4096), (4096, 14336)]
    bw, bwant = [], []
    for j, (m, n) in enumerate(shapes):
        p, a1, a2, _ = O.golden_case_inputs(m, n, 100 + j, {})
        bwant.append(orc.dequant_ref(p, a1, a2, m, n, O.BF16).view(np.int16).reshape(-1))
        bw.append((torch.from_numpy(p).to(dev), torch.from_numpy(a1).to(dev), torch.from_numpy(a2).to(dev),
                   torch.empty((m, n), dtype=torch.bfloat16, device=dev)))
    descs = (_lib.MatrixDesc * len(bw))(*[
        _lib.MatrixDesc(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(), o.data_ptr(),
                        o.shape[0], o.shape[1]) for (q, a1, a2, o) in bw])
    t0 = time.time()
    last_print = t0
    it = launches = checks = bad = 0
    while time.time() - t0 < args.seconds:
        for f in forms:
            f.launch(L, it, st)
        assert L.nf4_dequant_ref_batched(descs, len(bw), O.BF16, st) == 0
        launches += len(forms) + 1
        it += 1
        if it % args.check_every == 0:
            torch.cuda.synchronize()
            for f in forms:
                checks += 1
                if not f.check():
                    bad += 1
                    print(json.dumps({"mismatch": f.name, "iteration": it}), flush=True)
            for (q, a1, a2, o), w in zip(bw, bwant):
                checks += 1
                if not np.array_equal(o.view(torch.int16).cpu().numpy().reshape(-1), w):
                    bad += 1
                    print(json.dumps({"mismatch": f"batched {tuple(o.shape)}", "iteration": it}), flush=True)
        if time.time() - last_print > 30:
            last_print = time.time()
            print(json.dumps({"progress_s": round(last_print - t0), "iterations": it, "launches": launches,
                              "checks": checks, "mismatches": bad}), flush=True)
    torch.cuda.synchronize()
    print(json.dumps({"summary": {"seconds": round(time.time() - t0, 1), "iterations": it, "launches": launches,
                                  "checks": checks, "mismatches": bad, "forms": [f.name for f in forms] + ["batched"]}}),
          flush=True)


if __name__ == "__main__":
    main()
