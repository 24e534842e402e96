"""Per-wave phase timing of the flat dequant kernel (diagnostic build `make -C tools stamps`).

    python tools/flat_stamps.py [--shape 4096,4096] [--reps 8] [--flags 0] [--tile-dwords 4]

Each wave stamps s_memrealtime (100 MHz, 10 ns ticks) at entry, after its first
tile is decoded and its stores issued (= its first loads arrived), and at exit
after all its loads and stores completed; it also records the tiles it walked.
``--stream L`` (round 5): the same stamps for the last of L back-to-back launches in
bench.py's HBM-streamed regime, plus the boundary from the previous launch's last wave
exit to this launch's first wave entry.
Prints the launch-wide distributions (us, percentiles 0/10/50/90/100) relative
to the first wave's entry: wave entry (dispatch ramp), first-data latency
(first tile done - entry), exit, and the span (first entry -> last exit), next
to the HIP-event time of the same launches.  Buffers rotate over > 1 GiB so every
launch streams from HBM.
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
from nf4_triton_dequantization_amd import _lib  # noqa: E402


def pct(a):
    return [round(float(np.percentile(a, q)), 3) for q in (0, 10, 50, 90, 100)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4096,4096")
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--tile-dwords", type=int, default=4)
    ap.add_argument("--blocks-per-cu", type=int, default=0)
    ap.add_argument("--stream", type=int, default=0,
                    help="round 5: stamp the last of this many back-to-back launches (HBM-streamed "
                         "rotation, bench.py's regime) and the one before it, instead of cold single launches")
    args = ap.parse_args()
    if args.stream:
        return stream_main(args)
    # the diagnostic build beside the product one (the package import already
    # loaded libnf4dq.so); only the two entry points used here are bound
    L = ctypes.CDLL(os.path.join(REPO, "tools", "_build", "libnf4dq_stamps.so"))
    L.nf4_dequant_ref_cfg.restype = ctypes.c_int
    L.nf4_dequant_ref_cfg.argtypes = _lib.SIGNATURES["nf4_dequant_ref_cfg"][1]
    L.nf4_dbg_set_stamps.argtypes = [ctypes.c_void_p]
    L.nf4_dbg_set_stamps.restype = None
    dev = torch.device("cuda", 0)
    m, n = (int(v) for v in args.shape.split(","))
    nb = m * n // 64
    sets = max(4, (1 << 30) // (m * n * 5 // 2))
    ws = [(torch.randint(0, 256, (m * n // 2,), dtype=torch.uint8, device=dev),
           torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev),
           torch.rand((nb + 255) // 256, device=dev) * 0.01 + 1e-3,
           torch.empty((m, n), dtype=torch.bfloat16, device=dev)) for _ in range(sets)]
    max_waves = 1 << 20
    st = torch.zeros(max_waves * 4, dtype=torch.int64, device=dev)
    L.nf4_dbg_set_stamps(st.data_ptr())
    cfg = _lib.LaunchCfg(args.tile_dwords, args.blocks_per_cu, 1, args.flags)
    sp = torch.cuda.current_stream().cuda_stream
    rows, spans, evs = [], [], []
    for it in range(args.reps):
        q, a1, a2, o = ws[it % sets]
        st.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.nf4_dequant_ref_cfg(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                   o.data_ptr(), _lib.BF16, m, n, ctypes.byref(cfg), sp)
        e1.record()
        assert rc == 0, rc
        torch.cuda.synchronize()
        if it < 2:
            continue
        a = st.cpu().numpy().reshape(-1, 4)
        a = a[a[:, 0] > 0]
        t0 = a[:, 0].min()
        entry = (a[:, 0] - t0) / 100.0
        work = a[:, 3] > 0
        first = (a[work, 1] - a[work, 0]) / 100.0
        exit_ = (a[:, 2] - t0) / 100.0
        rows.append((entry, first, exit_, a[:, 3]))
        spans.append(exit_.max())
        evs.append(e0.elapsed_time(e1) * 1e3)
    agg = [np.concatenate([r[i] for r in rows]) for i in range(4)]
    print(json.dumps({"shape": [m, n], "flags": args.flags, "tile_dwords": args.tile_dwords,
                      "waves": int(len(rows[-1][0])), "tiles_per_wave": pct(agg[3]),
                      "span_us": pct(spans), "event_us": pct(evs), "entry_us": pct(agg[0]),
                      "first_tile_done_minus_entry_us": pct(agg[1]), "exit_us": pct(agg[2])}), flush=True)


def stream_main(args):
    """Back-to-back launches in bench.py's regime (>= 512 MiB of distinct reads and writes,
    inputs and outputs rotated independently): the last two launches of a run of
    ``--stream`` write their stamps to two buffers, so the boundary between them is seen
    from the waves' side (last wave exit of launch L-1 -> first wave entry of launch L)."""
    L = ctypes.CDLL(os.path.join(REPO, "tools", "_build", "libnf4dq_stamps.so"))
    L.nf4_dequant_ref.restype = ctypes.c_int
    L.nf4_dequant_ref.argtypes = _lib.SIGNATURES["nf4_dequant_ref"][1]
    L.nf4_dbg_set_stamps.argtypes = [ctypes.c_void_p]
    L.nf4_dbg_set_stamps.restype = None
    dev = torch.device("cuda", 0)
    m, n = (int(v) for v in args.shape.split(","))
    nb = m * n // 64
    n2 = (nb + 255) // 256
    pin = -(-(512 << 20) // (m * n // 2 + nb + 4 * n2))
    pout = -(-(512 << 20) // (2 * m * n))
    ins = [(torch.randint(0, 256, (m * n // 2,), dtype=torch.uint8, device=dev),
            torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev),
            torch.rand(n2, device=dev) * 0.01 + 1e-3) for _ in range(pin)]
    outs = [torch.empty((m, n), dtype=torch.bfloat16, device=dev) for _ in range(pout)]
    max_waves = 1 << 20
    bufs = [torch.zeros(max_waves * 4, dtype=torch.int64, device=dev) for _ in range(2)]
    sp = torch.cuda.current_stream().cuda_stream

    def launch(i, buf):
        q, a1, a2 = ins[i % pin]
        L.nf4_dbg_set_stamps(buf.data_ptr())
        rc = L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), nb, a2.data_ptr(), n2,
                               outs[i % pout].data_ptr(), _lib.BF16, m, n, sp)
        assert rc == 0, rc

    for i in range(max(pin, pout)):  # TLB-warm pass
        launch(i, bufs[0])
    torch.cuda.synchronize()
    rows = []
    for rep in range(args.reps):
        for b in bufs:
            b.zero_()
        torch.cuda._sleep(2_000_000)  # the host submits every launch while the device spins
        for i in range(args.stream):
            launch(i + rep * args.stream, bufs[(args.stream - 1 - i) % 2])  # the last launch -> bufs[0]
        torch.cuda.synchronize()
        last = bufs[0].cpu().numpy().reshape(-1, 4)
        prev = bufs[1].cpu().numpy().reshape(-1, 4)
        last = last[last[:, 0] > 0]
        prev = prev[prev[:, 0] > 0]
        t0 = last[:, 0].min()
        work = last[:, 3] > 0
        rows.append({"entry": (last[:, 0] - t0) / 100.0,
                     "first": (last[work, 1] - last[work, 0]) / 100.0,
                     "first_abs": (last[work, 1] - t0) / 100.0,
                     "exit": (last[:, 2] - t0) / 100.0,
                     "boundary": (t0 - prev[:, 2].max()) / 100.0,
                     "prev_span": (prev[:, 2].max() - prev[:, 0].min()) / 100.0})
    agg = {k: np.concatenate([np.atleast_1d(r[k]) for r in rows]) for k in rows[0]}
    print(json.dumps({"shape": [m, n], "mode": f"stream: last of {args.stream} back-to-back launches",
                      "in_sets": pin, "out_sets": pout, "waves": int(len(rows[-1]["entry"])),
                      "entry_us": pct(agg["entry"]), "first_tile_stored_minus_entry_us": pct(agg["first"]),
                      "first_tile_stored_us": pct(agg["first_abs"]), "exit_us": pct(agg["exit"]),
                      "span_us": pct([float(r["exit"].max()) for r in rows]),
                      "prev_launch_span_us": pct(agg["prev_span"]),
                      "boundary_prev_last_exit_to_first_entry_us": pct(agg["boundary"])}), flush=True)


if __name__ == "__main__":
    main()
