"""Measure the BASELINE.json configs other than the bench.py headline, on one GPU.

    python tools/bench_configs.py [--configs c3,c3b,c4,c5] [--reps 5] > profiles/r01/configs.jsonl

c3   Llama-3-8B: 32 layers x {q,o 4096x4096; k,v 1024x4096; gate,up 14336x4096;
     down 4096x14336} NF4->bf16, all 224 weights per pass through the batched
     C ABI (nf4_dequant_ref_batched, <= NF4DQ_BATCH_MAX matrices per launch).
c3b  the "4096/11008" shape set BASELINE names (Llama-2-7B: q,k,v,o 4096x4096;
     gate,up 11008x4096; down 4096x11008), same method.
c4   4096x4096 NF4 -> fp16 vs bf16 vs fp32 output, single launches over an
     independent input / output rotation (>= 512 MiB of distinct reads and of distinct
     writes, bench.py's HBM-streamed regime), timed as bench.py times its steps
     (eager, behind a device spin), the hipGraph replay beside it.
c5   one 8192x8192 NF4->bf16 matrix (the per-GPU unit of the 8-GPU config), the same
     rotation and method.
big  128256x8192 NF4->bf16 (Llama-3-70B lm_head size: 525 MB packed, past one buffer
     descriptor -- two row pieces in one launch).
odd  4096x4080 NF4->bf16: n % 64 != 0 (every row ends in a partial 64-block), so the
     matrix takes the chunk kernel (its dense form), not the flat kernel; same method as c4.
piece 4096x4090 NF4->bf16 and ->fp32, 4096x4100 NF4->bf16 (n % 8 != 0; a 4-element last
     block): the piece kernels (round 6), same method as c4, every output verified.
bnb  4096x4096 NF4->bf16 with bitsandbytes semantics (nf4_dequant_bnb: code2[A1] * A2
     + offset, flat blocks), same method as c4; its algorithmic bytes
     add the 1 KiB nested code book.

Every line: elements/s and algorithmic GB/s (SURVEY §8d bytes) vs the 8 TB/s
peak; timing = HIP events around the whole pass on the launch stream (c3/c3b: the
pass captured in a hipGraph, the eager figure alongside).  After timing, every
output the timed launches wrote is compared bit for bit with the C oracle
(``verified`` / ``verified_matrices`` in the line; a mismatch fails the run); the
oracle is pinned to the reference fallback at each of these shapes
(tests/golden/manifest.json C2/C3/C3b/C4/C5 digests).
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
from nf4_triton_dequantization_amd import _lib  # noqa: E402
import nf4_oracle as O  # noqa: E402  -- the checker of the timed outputs

_CORACLE = None


def verify(ws, code, bnb_code2=None, bnb_offset=0.0):
    """Every (q, a1, a2, out) output vs the C oracle on the same inputs; raises on a mismatch."""
    global _CORACLE
    if _CORACLE is None:
        _CORACLE = O.COracle()
        _CORACLE.set_threads(16)
    ocode = {_lib.F16: O.F16, _lib.BF16: O.BF16, _lib.F32: O.F32}[code]
    for i, (q, a1, a2, o) in enumerate(ws):
        m, n = o.shape
        hq, h1, h2 = q.cpu().numpy(), a1.cpu().numpy(), a2.cpu().numpy()
        if bnb_code2 is None:
            want = _CORACLE.dequant_ref(hq, h1, h2, m, n, ocode)
        else:
            want = _CORACLE.dequant_bnb(hq, h1, bnb_code2, h2, bnb_offset, m * n, ocode).reshape(m, n)
        wt = torch.from_numpy(want.view(np.int32 if code == _lib.F32 else np.int16)).to(o.device)
        got = o.view(torch.int32 if code == _lib.F32 else torch.int16)
        if not torch.equal(got, wt):
            raise AssertionError(f"output {i} ({m}x{n}) differs from the oracle")
    return len(ws)

PEAK = 8.0e12
LLAMA3_8B = [(4096, 4096), (1024, 4096), (1024, 4096), (4096, 4096), (14336, 4096), (14336, 4096), (4096, 14336)]
LLAMA2_7B = [(4096, 4096)] * 4 + [(11008, 4096), (11008, 4096), (4096, 11008)]


def alg_bytes(m, n, ob):
    N = m * n
    nb = N // 64
    n2 = (nb + 255) // 256
    g = ((n + 63) // 64 + 3) // 4
    return N // 2 + N * ob + nb + 4 * min(n2, m * g)


def make_weight(m, n, dev, gen, dt):
    nb = m * n // 64
    return (torch.randint(0, 256, (m * n // 2,), dtype=torch.uint8, device=dev, generator=gen),
            torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=gen),
            torch.rand((nb + 255) // 256, device=dev, generator=gen) * 0.01 + 1e-3,
            torch.empty((m, n), dtype=dt, device=dev))


def timed(fn, reps):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(reps):
        e0.record(st)
        fn()
        e1.record(st)
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) * 1e-3)
    best.sort()
    return best[len(best) // 2]


def run_model(name, shapes, layers, reps, dev):
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    ws = [make_weight(m, n, dev, gen, torch.bfloat16) for _ in range(layers) for (m, n) in shapes]
    descs = (_lib.MatrixDesc * len(ws))(*[
        _lib.MatrixDesc(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                        o.data_ptr(), o.shape[0], o.shape[1]) for (q, a1, a2, o) in ws])
    L = _lib.lib()

    def fn():
        rc = L.nf4_dequant_ref_batched(descs, len(ws), _lib.BF16, torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc

    te = timed(fn, reps)  # eager: host launches inside the timed region
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    t = timed(g.replay, reps)  # the pass captured once (as bench.py times its steps)
    elems = sum(o.numel() for *_, o in ws)
    byt = sum(alg_bytes(o.shape[0], o.shape[1], 2) for *_, o in ws)
    launches = -(-len(ws) // _lib.BATCH_MAX)
    checked = verify(ws, _lib.BF16)
    return {"config": name, "verified": True, "verified_matrices": checked, "matrices": len(ws), "launches": launches, "elements": elems, "seconds": t,
            "elements_per_s": elems / t, "algorithmic_bytes": byt, "GBps": byt / t / 1e9, "frac": byt / t / PEAK,
            "timing": "hipGraph replay of the pass", "eager_seconds": te, "eager_frac": byt / te / PEAK}


def eager_per_launch(launch, steps, reps):
    """bench.py's timing: a device spin covering the host's submission, 8 untimed lead
    launches, then `steps` launches between HIP events on the launch stream; median
    over `reps` of the per-launch time (s)."""
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    torch.cuda._sleep(2_000_000)
    e1.record(st)
    torch.cuda.synchronize()
    cyc_per_us = 2_000_000 / max(e0.elapsed_time(e1) * 1e3, 1.0)
    ts = []
    for _ in range(reps):
        torch.cuda._sleep(int(cyc_per_us * (40.0 * (steps + 8) + 200.0)))
        for j in range(8):
            launch(j - 8)
        e0.record(st)
        for i in range(steps):
            launch(i)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3 / steps)
    ts.sort()
    return ts[len(ts) // 2]


MIN_READ_FOOTPRINT = 512 << 20  # bench.py's HBM-streamed rotation (DESIGN.md "cache regime")
MIN_WRITE_FOOTPRINT = 512 << 20


def rotation(m, n, ob, extra_read=0):
    """(input sets, output sets): >= 512 MiB of distinct reads and of distinct writes,
    as bench.rotation_sets -- every launch reads its packed weight from HBM."""
    rd = m * n // 2 + m * n // 64 + 4 * ((m * n // 64 + 255) // 256) + extra_read
    wr = m * n * ob
    return max(1, -(-MIN_READ_FOOTPRINT // rd)), max(1, -(-MIN_WRITE_FOOTPRINT // wr))


def rotating_sets(m, n, dt, dev, gen, pin, pout):
    """pin (packed, absmax, absmax2) input sets and pout output buffers."""
    ins = [make_weight(m, n, dev, gen, dt)[:3] for _ in range(pin)]
    outs = [torch.empty((m, n), dtype=dt, device=dev) for _ in range(pout)]
    return ins, outs


def last_writes(pin, pout, steps, limit=4):
    """(input set, output set) of the last timed launch that wrote each of the first
    `limit` output sets: what the outputs hold when the timing ends."""
    res = []
    for j in range(min(pout, steps, limit)):
        i = j + ((steps - 1 - j) // pout) * pout
        res.append((i % pin, j))
    return res


def run_single(name, m, n, dt, code, reps, dev, steps=64):
    """Single launches over an independent input / output rotation (step i reads input
    set i % Pin, writes output set i % Pout; >= 512 MiB distinct reads and writes, the
    regime of bench.py's headline).  Timed as bench.py times its steps (eager launches
    behind a spin, ``us_per_launch``); the hipGraph replay of the same launches is
    reported beside it (``graph_us_per_launch``): on ROCm 7.2 a replay adds 1-3 us per
    8192^2 kernel, as a system-scope release between eager launches does
    (tools/c5_probe.py, profiles/r03/c5/)."""
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    ob = torch.empty((), dtype=dt).element_size()
    pin, pout = rotation(m, n, ob)
    ins, outs = rotating_sets(m, n, dt, dev, gen, pin, pout)
    L = _lib.lib()

    def launch(i):
        q, a1, a2 = ins[i % pin]
        o = outs[i % pout]
        assert L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                 o.data_ptr(), code, m, n, torch.cuda.current_stream().cuda_stream) == 0

    for i in range(max(pin, pout)):  # every set touched once (TLB-warm, as resident weights are)
        launch(i)
    torch.cuda.synchronize()
    t = eager_per_launch(launch, steps, reps)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for i in range(steps):
            launch(i)
    tg = timed(graph.replay, reps) / steps
    byt = alg_bytes(m, n, ob)
    checked = verify([ins[a] + (outs[b],) for a, b in last_writes(pin, pout, steps)], code)
    rd = pin * (m * n // 2 + m * n // 64 + 4 * ((m * n // 64 + 255) // 256))
    return {"config": name, "verified": True, "verified_matrices": checked, "m": m, "n": n,
            "out_dtype": str(dt).replace("torch.", ""), "in_sets": pin, "out_sets": pout,
            "read_footprint_bytes": rd, "write_footprint_bytes": pout * m * n * ob,
            "weights_from": "HBM (distinct reads >= 512 MiB)" if rd >= MIN_READ_FOOTPRINT else "Infinity Cache possible",
            "us_per_launch": t * 1e6, "elements_per_s": m * n / t, "algorithmic_bytes": byt, "GBps": byt / t / 1e9,
            "frac": byt / t / PEAK, "timing": "eager launches behind a spin (bench.py's method)",
            "graph_us_per_launch": tg * 1e6, "graph_frac": byt / tg / PEAK}


def run_bnb(name, m, n, reps, dev, steps=64):
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    pin, pout = rotation(m, n, 2)
    ins, outs = rotating_sets(m, n, torch.bfloat16, dev, gen, pin, pout)
    code2 = torch.linspace(-1, 1, 256, device=dev, dtype=torch.float32)
    L = _lib.lib()
    numel = m * n

    def launch(i):
        q, a1, a2 = ins[i % pin]
        assert L.nf4_dequant_bnb(q.data_ptr(), a1.data_ptr(), a1.numel(), code2.data_ptr(), a2.data_ptr(),
                                 a2.numel(), ctypes.c_float(0.0123), outs[i % pout].data_ptr(), _lib.BF16, numel,
                                 64, 256, torch.cuda.current_stream().cuda_stream) == 0

    for i in range(max(pin, pout)):
        launch(i)
    torch.cuda.synchronize()
    t = eager_per_launch(launch, steps, reps)
    for i in range(steps):  # the outputs the checker reads: the same launches in order
        launch(i)
    nb = numel // 64
    byt = numel // 2 + 2 * numel + nb + 4 * ((nb + 255) // 256) + 1024
    checked = verify([ins[a] + (outs[b],) for a, b in last_writes(pin, pout, steps)], _lib.BF16,
                     bnb_code2=code2.cpu().numpy(), bnb_offset=np.float32(0.0123))
    return {"config": name, "verified": True, "verified_matrices": checked, "m": m, "n": n, "out_dtype": "bfloat16",
            "in_sets": pin, "out_sets": pout, "us_per_launch": t * 1e6,
            "elements_per_s": numel / t, "algorithmic_bytes": byt, "GBps": byt / t / 1e9, "frac": byt / t / PEAK,
            "timing": "eager launches behind a spin (bench.py's method)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c3b,c4,c5,big,odd,piece,bnb")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--layers", type=int, default=32)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    todo = args.configs.split(",")
    if "c3" in todo:
        print(json.dumps(run_model("c3 Llama-3-8B linears x32 NF4->bf16 batched", LLAMA3_8B, args.layers, args.reps,
                                   dev)), flush=True)
        torch.cuda.empty_cache()
    if "c3b" in todo:
        print(json.dumps(run_model("c3b Llama-2-7B (4096/11008) linears x32 NF4->bf16 batched", LLAMA2_7B,
                                   args.layers, args.reps, dev)), flush=True)
        torch.cuda.empty_cache()
    if "c4" in todo:
        for dt, code in ((torch.float16, _lib.F16), (torch.bfloat16, _lib.BF16), (torch.float32, _lib.F32)):
            print(json.dumps(run_single("c4 4096x4096 dtype sweep", 4096, 4096, dt, code, args.reps, dev)),
                  flush=True)
        torch.cuda.empty_cache()
    if "c5" in todo:
        print(json.dumps(run_single("c5 8192x8192 per-GPU unit", 8192, 8192, torch.bfloat16, _lib.BF16, args.reps, dev)),
              flush=True)
        torch.cuda.empty_cache()
    if "big" in todo:
        print(json.dumps(run_single("big 128256x8192 (a 70B lm_head: two flat pieces, one launch)", 128256, 8192,
                                    torch.bfloat16, _lib.BF16, args.reps, dev, steps=8)), flush=True)
        torch.cuda.empty_cache()
    if "odd" in todo:
        print(json.dumps(run_single("odd 4096x4080 (n % 64 != 0: the chunk kernel)", 4096, 4080, torch.bfloat16,
                                    _lib.BF16, args.reps, dev)), flush=True)
        torch.cuda.empty_cache()
    if "piece" in todo:
        for n, dt, code in ((4090, torch.bfloat16, _lib.BF16), (4090, torch.float32, _lib.F32),
                            (4100, torch.bfloat16, _lib.BF16)):
            print(json.dumps(run_single(f"piece 4096x{n} (n % 8 != 0: the piece kernel)", 4096, n, dt, code,
                                        args.reps, dev)), flush=True)
        torch.cuda.empty_cache()
    if "bnb" in todo:
        print(json.dumps(run_bnb("bnb-semantics 4096x4096 NF4->bf16", 4096, 4096, args.reps, dev)), flush=True)


if __name__ == "__main__":
    main()
