"""Where does the 8192^2 single-launch time go?  (C5's per-rank unit; diagnostic)

One process, the same kernel (nf4_dequant_ref, 8192x8192 NF4->bf16), 8 rotating
buffer sets (1.3 GB >> the 256 MiB Infinity Cache), crossed over:

* layout   -- ``interleaved``: per set q, a1, a2, out allocated in turn (what
              tools/bench_configs.py does); ``separate``: all q, all out, then all
              a1, all a2 (tools/value_sensitivity.py); ``slab``: like separate,
              but the 8 absmax byte arrays are 2 MiB-aligned slices of one
              allocation; ``shared``: one a1/a2 pair for every set (content
              resident in the Infinity Cache after the first launch)
* method   -- ``graph``: 32 launches captured once, median of 5 replays (as
              bench_configs); ``eager``: a device spin covering the host's
              submission, 8 untimed lead launches, then 32 timed launches between
              HIP events on the launch stream (as bench.py); ``eager+event``: the
              same with a default HIP event recorded after every launch (a
              system-scope release between kernels)

Prints one JSON line per (round, layout, method): us per launch and fraction of
the 8 TB/s peak for the SURVEY §8d algorithmic bytes (168,837,120 B).
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tools")]
from nf4_triton_dequantization_amd import _lib  # noqa: E402
from hbm_ceiling import graph_time  # noqa: E402

PEAK = 8e12
M = N = 8192
P = 8
STEPS = 32
NBYTES, NB = M * N // 2, M * N // 64
N2 = (NB + 255) // 256
ALG = NBYTES + 2 * M * N + NB + 4 * N2
L = _lib.lib()
dev = torch.device("cuda", 0)


def rnd_u8(n, g):
    return torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev, generator=g)


def rnd_a2(g):
    return torch.rand(N2, device=dev, generator=g) * 0.01 + 1e-3


def make(layout, seed):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    if layout == "interleaved":
        sets = []
        for _ in range(P):
            q = rnd_u8(NBYTES, g)
            a1 = rnd_u8(NB, g)
            a2 = rnd_a2(g)
            out = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
            sets.append((q, a1, a2, out))
        return sets, None
    qs = [rnd_u8(NBYTES, g) for _ in range(P)]
    outs = [torch.empty((M, N), dtype=torch.bfloat16, device=dev) for _ in range(P)]
    keep = None
    if layout == "separate":
        a1s = [rnd_u8(NB, g) for _ in range(P)]
    elif layout == "slab":
        keep = torch.empty(P * (2 << 20) + (2 << 20), dtype=torch.uint8, device=dev)
        base = (-keep.data_ptr()) % (2 << 20)  # first 2 MiB boundary inside the slab
        a1s = [keep[base + i * (2 << 20): base + i * (2 << 20) + NB] for i in range(P)]
        for a in a1s:
            a.copy_(rnd_u8(NB, g))
    else:  # shared
        a1s = [rnd_u8(NB, g)] * P
    a2s = [rnd_a2(g) for _ in range(P)] if layout != "shared" else [rnd_a2(g)] * P
    return list(zip(qs, a1s, a2s, outs)), keep


def launcher(sets):
    def step(i):
        q, a1, a2, o = sets[i % P]
        rc = L.nf4_dequant_ref(q.data_ptr(), NBYTES, a1.data_ptr(), NB, a2.data_ptr(), N2, o.data_ptr(), _lib.BF16,
                               M, N, torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
    return step


def eager_time(step, steps, reps=5, fence_each=False):
    st = torch.cuda.current_stream()
    # spin rate of torch.cuda._sleep on this device
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
            step(j - 8)
        e0.record(st)
        for i in range(steps):
            step(i)
            if fence_each:
                # a default (non-timing) event: recording it is a system-scope release
                # (L2 write-back) after every launch -- what a graph node may carry
                torch.cuda.Event().record(st)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3 / steps)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    layouts = sys.argv[1].split(",") if len(sys.argv) > 1 else ["interleaved", "separate", "slab", "shared"]
    built = {}
    for k, lay in enumerate(layouts):
        built[lay] = make(lay, 11 + k)
        step = launcher(built[lay][0])
        for i in range(2 * P):  # every set touched (TLB-warm, as resident weights are)
            step(i)
    torch.cuda.synchronize()
    for r in range(3):
        for lay in layouts:
            step = launcher(built[lay][0])
            for meth in ("graph", "eager", "eager+event"):
                t = (graph_time(step, STEPS) if meth == "graph" else
                     eager_time(step, STEPS, fence_each=meth == "eager+event"))
                print(json.dumps({"round": r, "layout": lay, "method": meth, "us": round(t * 1e6, 3),
                                  "frac": round(ALG / t / PEAK, 4)}), flush=True)


if __name__ == "__main__":
    main()
