"""Benchmark: NF4 -> bf16 double dequantization of a 4096x4096 weight on MI355X.

Metric (BASELINE.json): dequantized elements/s + achieved HBM GB/s, 4096x4096
NF4->bf16 (configs[1]).  A *step* is one dequantization of one 4096x4096
weight through the product C ABI (``nf4_dequant_ref``), inputs resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Timed region (the ``value``): K steps captured once into a hipGraph and
replayed, bracketed by barrier + synchronize on both sides; step i reads and
writes buffer set i % P, with P sets (P * 42 MB >> the 256 MiB Infinity Cache)
so every step streams from and to HBM.  ``value`` = elements of all ranks / max
over ranks of the region time.

Roofline (``roofline``): ``achieved`` = algorithmic bytes per launch (SURVEY
§8d: N/2 packed + 2N out + nb absmax + 4*min(n2, m*G) nested absmax) / mean
launch duration, the latter from the HIP events that bracket the timed region
on the launch stream (region time / K: inter-launch gaps count against us);
``peak`` = 8 TB/s; ``traffic`` = PMC-counted HBM bytes per launch from
profiles/<round>/pmc_traffic.json (tools/pmc_traffic.py) when present.

CPU baseline (``cpu_baseline``, rank 0 at N=1), same 4096x4096 workload on this
GPU's host share of cores (at most 16): ``value`` = oracle/fallback_torch.py, a
torch-CPU restatement with the reference fallback's loop structure (the CPU path
the reference itself runs); ``native`` = the C oracle over OpenMP threads;
``single_thread`` = the C oracle on one thread.

Multi-GPU (weak scaling): every rank dequantizes its own matrices; rank 0 owns
the quant statistics of all ranks' matrices and broadcasts them once over RCCL
at setup (sharding.broadcast_quant_stats) -- no collective on the data path.
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
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from nf4_triton_dequantization_amd import _lib  # noqa: E402
from nf4_triton_dequantization_amd.sharding import QuantStats, broadcast_quant_stats, max_over_ranks  # noqa: E402

PEAK_HBM = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md)
ROUND = "r01"


def algorithmic_bytes(m: int, n: int, out_bytes: int, nb: int, n2: int) -> int:
    """packed + output + u8 absmax + unique fp32 nested absmax."""
    N = m * n
    bpr = (n + 63) // 64
    groups = (bpr + 3) // 4
    return N // 2 + N * out_bytes + nb + 4 * min(n2, m * groups)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def gen_set(m, n, seed, rank):
    """Packed weight for (rank, set) from the shared splitmix64 generator."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import nf4_oracle as O  # input generator (deterministic); not on the measured path

    return O.splitmix64_bytes(seed * 1000003 + rank, m * n // 2, stream=1)


def gen_stats(m, n, seed):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import nf4_oracle as O

    nb = (m * n + 63) // 64
    n2 = (nb + 255) // 256
    return O.splitmix64_bytes(seed, nb, stream=2), O.uniform_f32(seed, n2, 1e-3, 1e-2, stream=3)


def cpu_baseline(m, n, seconds, dtype_code):
    """CPU figures on the same workload, on this GPU's host share of cores (<= 16):

    * ``value``: oracle/fallback_torch.py -- torch-CPU restatement with the
      reference fallback's execution shape (kernel_optimized.py:208-314: per-block
      scale loop, per-column strided writes), the "reference fallback" row of
      BASELINE.md's CPU plan; ~`seconds` of repeats;
    * ``native``: the C oracle, rows over OpenMP threads (~`seconds`/2);
    * ``single_thread``: the C oracle on one thread (~`seconds`/4).
    """
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import fallback_torch as F
    import nf4_oracle as O

    c = O.COracle()
    p, a1, a2 = O.make_inputs(m, n, 3409)
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1))

    def repeat(fn, secs):
        fn()  # warm (page-in, thread pool)
        t0 = time.perf_counter()
        reps = 0
        while True:
            fn()
            reps += 1
            el = time.perf_counter() - t0
            if el >= secs:
                return reps, el

    tdt = torch.bfloat16 if dtype_code == O.BF16 else torch.float16
    tp, ta1, ta2 = torch.from_numpy(p), torch.from_numpy(a1), torch.from_numpy(a2)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        rf, ef = repeat(lambda: F.dequant_fallback(tp, ta1, ta2, m, n, tdt), seconds)
    finally:
        torch.set_num_threads(prev)

    def native(nthreads, secs):
        c.set_threads(nthreads)
        return repeat(lambda: c.dequant_ref(p, a1, a2, m, n, dtype_code), secs)

    rn, en = native(threads, max(1.0, seconds / 2))
    r1, e1 = native(1, max(1.0, seconds / 4))
    c.set_threads(1)
    dname = "bf16" if dtype_code == O.BF16 else "fp16"
    return {"value": rf * m * n / ef, "unit": "elements/s", "cores": threads, "kind": "port",
            "sample": f"{rf} x {m}x{n} NF4->{dname} by oracle/fallback_torch.py (the reference fallback's "
                      f"loop structure in torch-CPU, {threads} threads), {ef:.1f} s",
            "native": {"value": rn * m * n / en, "cores": threads,
                       "sample": f"{rn} x {m}x{n} by oracle/nf4_oracle.c (scalar C, rows over {threads} "
                                 f"OpenMP threads), {en:.1f} s"},
            "single_thread": {"value": r1 * m * n / e1, "cores": 1,
                              "sample": f"{r1} x {m}x{n} by oracle/nf4_oracle.c, 1 thread, {e1:.1f} s"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16"])
    ap.add_argument("--sets", type=int, default=16, help="rotating buffer sets (>256 MiB total)")
    ap.add_argument("--streams", type=int, default=1, help="streams the steps round-robin over")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--tile-dwords", type=int, default=4)
    ap.add_argument("--blocks-per-cu", type=int, default=0)
    ap.add_argument("--nontemporal", type=int, default=1)
    ap.add_argument("--flags", type=int, default=0, help="NF4DQ_CFG_* bits (1 = nt loads)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) for real runs; gloo to rehearse")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal on a box with fewer GPUs than ranks (gloo only): ranks share devices
    ndev = torch.cuda.device_count()
    local_dev = local if args.dist_backend == "nccl" else local % max(1, ndev)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    m, n, P = args.m, args.n, args.sets
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    code = _lib.BF16 if args.dtype == "bf16" else _lib.F16
    L = _lib.lib()

    # ---- setup: resident inputs, quant stats broadcast from rank 0 ----------
    t_setup = time.perf_counter()
    if rank == 0:
        stats = []
        for r in range(world):
            for s in range(P):
                a1, a2 = gen_stats(m, n, 3409 + 7919 * r + s)
                stats.append(QuantStats(m, n, torch.from_numpy(a1), torch.from_numpy(a2), dt))
    else:
        stats = None
    if world > 1:
        torch.cuda.synchronize()
        tb = time.perf_counter()
        stats = broadcast_quant_stats(stats, dev, src=0)
        torch.cuda.synchronize()
        bcast_ms = (time.perf_counter() - tb) * 1e3
    else:
        stats = [QuantStats(s.m, s.n, s.absmax.to(dev), s.absmax2.to(dev), s.dtype) for s in stats]
        bcast_ms = 0.0
    mine = stats[rank * P:(rank + 1) * P]
    sets = []
    for s in range(P):
        q = torch.from_numpy(gen_set(m, n, 3409 + s, rank)).to(dev)
        out = torch.empty((m, n), dtype=dt, device=dev)
        sets.append((q, mine[s].absmax, mine[s].absmax2, out))
    torch.cuda.synchronize()
    log(f"[rank {rank}] setup {time.perf_counter() - t_setup:.1f}s, quant_state broadcast {bcast_ms:.2f} ms")

    cfg = _lib.LaunchCfg(args.tile_dwords, args.blocks_per_cu, args.nontemporal, args.flags)
    cfg_p = ctypes.byref(cfg)

    def launch(i, stream_ptr):
        q, a1, a2, out = sets[i % P]
        rc = L.nf4_dequant_ref_cfg(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                   out.data_ptr(), code, m, n, cfg_p, stream_ptr)
        if rc:
            raise RuntimeError(f"nf4_dequant_ref_cfg: {_lib.strerror(rc)}")

    main_stream = torch.cuda.current_stream(dev)
    side = [torch.cuda.Stream(dev) for _ in range(max(0, args.streams - 1))]

    def issue(k0, count):
        """Steps k0..k0+count-1 round-robin over main + side streams."""
        if not side:
            ptr = torch.cuda.current_stream(dev).cuda_stream
            for i in range(k0, k0 + count):
                launch(i, ptr)
            return
        cur = torch.cuda.current_stream(dev)
        streams = [cur] + side
        for s in side:
            s.wait_stream(cur)
        for i in range(k0, k0 + count):
            launch(i, streams[i % len(streams)].cuda_stream)
        for s in side:
            cur.wait_stream(s)

    # correctness sanity of set 0 against the oracle (the tests do the full job)
    issue(0, 1)
    torch.cuda.synchronize()
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import nf4_oracle as O

    q0, a10, a20, o0 = sets[0]
    rows = slice(0, 64)
    want = O.dequant_ref_np(q0[: 64 * n // 2].cpu().numpy(), a10.cpu().numpy(), a20.cpu().numpy(), 64, n,
                            O.BF16 if args.dtype == "bf16" else O.F16)
    got = o0[rows].contiguous().view(torch.int16).cpu().numpy().view(np.uint16)
    if not np.array_equal(got, want):
        raise RuntimeError("bench sanity check failed: HIP output differs from the oracle")

    # ---- warmup + graph capture ----------------------------------------------
    for w in range(args.warmup):
        issue(w, 1)
    torch.cuda.synchronize()
    graph = None
    if not args.no_graph:
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                issue(0, args.steps)
            graph.replay()  # upload + one untimed pass
            torch.cuda.synchronize()
        except Exception as e:  # capture unsupported -> eager issue, reported in config
            log(f"[rank {rank}] hipGraph capture failed ({e}); timing eager launches")
            graph = None
            torch.cuda.synchronize()

    # ---- timed region -----------------------------------------------------------
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0.record(main_stream)
    if graph is not None:
        graph.replay()
    else:
        issue(0, args.steps)
    ev1.record(main_stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_ms = ev0.elapsed_time(ev1)
    if world > 1:
        t_ms = max_over_ranks(t_ms, dev)

    # ---- roofline: mean launch duration = HIP-event time of the timed region / K
    # (events on the launch stream; includes the inter-launch gaps, so it is an
    # upper bound on the rocprof per-kernel duration committed under profiles/).
    kt_mean = t_ms * 1e3 / args.steps  # us

    out_b = 2
    nb, n2 = sets[0][1].numel(), sets[0][2].numel()
    alg = algorithmic_bytes(m, n, out_b, nb, n2)
    achieved = alg / (kt_mean * 1e-6)
    traffic = None
    pmc_path = os.path.join(REPO, "profiles", ROUND, "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            if pmc.get("m") == m and pmc.get("n") == n and pmc.get("dtype") == args.dtype:
                traffic = pmc.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    elems = m * n * args.steps * world
    value = elems / (t_ms * 1e-3)
    res = {
        "metric": "dequantized elements/s (4096x4096 NF4->bf16, blocksize 64 / nested 256)",
        "value": value,
        "unit": "elements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_ms / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (splitmix64 packed weights + absmax, resident in HBM)",
        "hbm_gb_s": value * alg / (m * n) / 1e9,
        "config": {
            "workload": f"{m}x{n} NF4->{args.dtype} double dequant (BASELINE configs[1]), one matrix per step",
            "m": m, "n": n, "out_dtype": args.dtype, "arith": "u8 unpack, fp32 scale/multiply, RNE to bf16",
            "buffer_sets": P, "launch": "hipGraph" if graph is not None else "eager",
            "streams": args.streams, "tile_dwords": args.tile_dwords, "blocks_per_cu": args.blocks_per_cu,
            "nontemporal": args.nontemporal, "flags": args.flags, "parallelism": f"shard{world} (independent matrices)",
            "quant_state_broadcast_ms": round(bcast_ms, 3), "dist_backend": args.dist_backend if world > 1 else None,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved / 1e9,
            "peak": PEAK_HBM / 1e9,
            "unit": "GB/s",
            "frac": achieved / PEAK_HBM,
            "traffic": traffic,
            "kernel": "nf4_flat_kernel",
            "launch_us_mean": kt_mean,
            "launch_us_source": "HIP events over the timed region / steps (gaps included)",
            "algorithmic_bytes_per_launch": alg,
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(m, n, args.cpu_seconds, O.BF16 if args.dtype == "bf16" else O.F16)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
