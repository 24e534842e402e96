"""The headline's launches spread over S HIP streams (tools only; not the bench.py metric).

    python tools/multistream_probe.py [--streams 1,2,3,4] [--steps 128] [--rounds 7]

benchmark.py (the reference harness, :68-84) dequantizes three weights concurrently on
three streams.  This probe times K = --steps 4096^2 NF4 -> bf16 launches of the drop-in C
ABI (nf4_dequant_ref) over bench.py's HBM-streamed rotation (63 input / 16 output sets),
issued round-robin on S streams with no dependencies between them: every stream waits
on one gate event recorded after a device spin on stream 0 (so the host's submission
is hidden, as in bench.py), and stream 0 waits for the others' last launches before the
end event.  S = 1 is bench.py's method.  With S > 1 a launch can start while the
previous one drains, so the per-launch time shows how much of a dependent launch the
boundary between launches costs.  One JSON line per S: median / min / max us per launch
and the fraction of 8 TB/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from nf4_triton_dequantization_amd import _lib  # noqa: E402
from bench_configs import PEAK, alg_bytes, rotating_sets, rotation  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,2,3,4")
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=7)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    m = n = 4096
    pin, pout = rotation(m, n, 2)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    ins, outs = rotating_sets(m, n, torch.bfloat16, dev, gen, pin, pout)
    s0 = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s0)
    torch.cuda._sleep(2_000_000)
    e1.record(s0)
    torch.cuda.synchronize()
    cyc_per_us = 2_000_000 / max(e0.elapsed_time(e1) * 1e3, 1.0)
    counts = [int(v) for v in args.streams.split(",")]
    pool = [s0] + [torch.cuda.Stream() for _ in range(max(counts) - 1)]

    def launch(i, st):
        q, a1, a2 = ins[i % pin]
        o = outs[i % pout]
        rc = L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                               o.data_ptr(), _lib.BF16, m, n, st.cuda_stream)
        assert rc == 0, rc

    for i in range(max(pin, pout)):
        launch(i, s0)
    torch.cuda.synchronize()
    res = {S: [] for S in counts}
    for _ in range(args.rounds):
        for S in counts:
            streams = pool[:S]
            gate = torch.cuda.Event()
            torch.cuda._sleep(int(cyc_per_us * (40.0 * (args.steps + 8) + 200.0)))
            for j in range(8):  # lead launches on stream 0
                launch(j - 8, s0)
            e0.record(s0)
            gate.record(s0)
            for st in streams[1:]:
                st.wait_event(gate)
            for i in range(args.steps):
                launch(i, streams[i % S])
            for st in streams[1:]:
                done = torch.cuda.Event()
                done.record(st)
                s0.wait_event(done)
            e1.record(s0)
            torch.cuda.synchronize()
            res[S].append(e0.elapsed_time(e1) * 1e3 / args.steps)
    byt = alg_bytes(m, n, 2)
    for S in counts:
        ts = sorted(res[S])
        med = ts[len(ts) // 2]
        print(json.dumps({"streams": S, "steps": args.steps, "rounds": args.rounds, "in_sets": pin, "out_sets": pout,
                          "us_per_launch_median": round(med, 3), "us_min": round(ts[0], 3), "us_max": round(ts[-1], 3),
                          "frac": round(byt / (med * 1e-6) / PEAK, 4)}), flush=True)


if __name__ == "__main__":
    main()
