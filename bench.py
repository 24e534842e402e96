"""Benchmark: NF4 double dequantization on MI355X (BASELINE.json metric).

Metric (BASELINE.json): dequantized elements/s + achieved HBM GB/s, 4096x4096
NF4->bf16 (configs[1]).  A *step* is one pass of the hot path over one batch:

* ``--workload c2`` (default; the headline): one 4096x4096 NF4->bf16 weight per
  rank through the C ABI (``nf4_dequant_ref``); weak scaling (each rank its own
  matrix);
* ``--workload c5`` (BASELINE configs[4]): the 8 independent 8192x8192 matrices,
  split round-robin over the ranks (one per GPU at N=8), each rank's share in one
  batched launch (``nf4_dequant_ref_batched``); strong scaling (the 8-matrix job
  is fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

``--gpus N`` without a launcher (WORLD_SIZE unset) spawns N fresh rank processes
before this process touches the GPU and relays rank 0's line; under a launcher
WORLD_SIZE must equal N.

Timed regions (``value``): R = ``--repeats`` (default 7) regions of exactly K steps,
each K eager launches of the product C-ABI entry (``nf4_dequant_ref``, arguments
prepared up front), bracketed by barrier + synchronize on both sides, HIP events on the
launch stream around them.  Per region the max over ranks counts; the region with the
median of those maxima is the result (median, not one sample), and every
region's figure is on the line (``repeats``).  Ahead of each start event sit L = 16
untimed launches of the preceding buffer sets, so the queue holds real work when
timing starts, as in a steady stream of weights, and ahead of those a device spin that
outlasts the host's submission of all L + K launches (``--lead spin-steps``): the K
kernels then run back to back even when a profiler's per-dispatch interception makes
the host slower than the GPU (a kernel trace without it showed host-bound gaps and
per-kernel times 11 % above the events' figure); before that, one untimed launch per
buffer set warms the GPU TLB for every set.  ``--launch graph`` captures the K steps
into one hipGraph instead: on ROCm 7.2 a replay carries a fixed ~7-10 us outside the
kernels (rocprof: 20 launches span 139 us, the events 149 us), 0.4-0.5 us per step at
the driver's K = 20 (A/B: profiles/r02/bench_eager_ab.txt).  Step i uses input set
i % Pin and output set i % Pout, rotated independently: Pin so that each rank's
distinct READ bytes (packed weights + statistics) span >= 512 MiB -- 2x the 256 MiB
Infinity Cache, so every weight comes from HBM as in a model pass
(profiles/r04/cache/cache_ab_4096.jsonl: the launch time depends on the distinct reads
only; below ~256 MB the weights are re-read from the Infinity Cache) -- and Pout so
that the outputs span >= 512 MiB; under graph replay Pin also keeps a set's reuse
>= 512 MiB of reads apart across the untimed -> timed boundary (a scratch-write flush
instead costs 1-2 us per step through TLB misses, profiles/r02/bench_ab.txt).
``value`` = elements of all ranks / the median region's time.

Roofline (``roofline``): ``achieved`` = algorithmic bytes per launch (SURVEY
§8d: N/2 packed + 2N out + nb absmax + 4*min(n2, m*G) nested absmax) / launch
duration = HIP-event time of the median region on the launch stream / K
(inter-launch gaps count against us; min / median / max over the regions beside it);
``peak`` = 8 TB/s; ``traffic`` = PMC-counted HBM bytes per launch from
profiles/<round>/pmc_traffic.json (tools/pmc_traffic.py) when present for this shape.
``twin``: the memory-system twin of the same launch (the flat kernel's loads and
stores over the same one-tile-per-wave grid, no decode, no scale gathers:
tools/stream_probe.hip twin_mix), timed right after the headline by the same method on
the same rotation.  A reference point, NOT a ceiling: the product is faster than it
(``kernel_over_twin`` < 1; the scale gathers change how the loads and nt stores
interleave), so it bounds nothing.  ``measured_copy_peak``: the
guide's measured float4-copy rate (6.29 TB/s, MI355X_MICROARCH.md) beside the 8 TB/s
spec, and ``frac_of_measured_copy`` the headline against it.

CPU baseline (``cpu_baseline``, rank 0 at N=1), same workload on this GPU's
host share of cores (at most 16): ``value`` = oracle/fallback_torch.py, a
torch-CPU restatement with the reference fallback's loop structure (the CPU path
the reference itself runs, bit-equal to it); ``native`` = this library's own
host path ``nf4_dequant_ref_cpu`` (AVX2, same threads); ``single_thread`` = the
same at 1 thread.

``--backend cpu`` runs the steps through ``nf4_dequant_ref_cpu`` on host memory
(wall-clock timing, no roofline): the rehearsal mode the CPU tests use to drive
the spawn / gloo / max-over-ranks path without a GPU.

Multi-GPU: every rank dequantizes its own matrices; rank 0 owns the quant
statistics of every rank's matrices and scatters them once over RCCL at setup, each
rank receiving only its own matrices' statistics (sharding.scatter_quant_stats, timed
and reported separately as ``quant_state_scatter_ms``) -- no collective on the data
path.  ``--dist-backend nccl`` at N = 1 forms a one-rank group, so the scatter runs
over RCCL on a single GPU as well.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_HBM = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md)
MEASURED_COPY = 6.29e12  # B/s, the guide's measured float4 copy (MI355X_MICROARCH.md: 79 % of spec)
ROUNDS = ("r06", "r05", "r04", "r03", "r02", "r01")  # profiles/<round>/pmc_traffic.json, newest first
# Rotation (round 4, profiles/r04/cache/cache_ab_4096.jsonl): input sets (packed weight +
# absmax + nested absmax) and output sets rotate independently.  The per-launch time
# depends on the distinct READ bytes only: at 4096^2 6.89 us while they stay <= 225 MB
# (the packed weights are then read from the 256 MiB Infinity Cache -- the nt output
# stores do not displace them), 7.4 us at 268 MB, 7.9-8.0 us from 346 MB to 1 GB; the
# written bytes change nothing from 67 MB to 2 GB.  A streamed model's weights are read
# once per pass, so the headline rotates >= 512 MiB of distinct input bytes per rank
# (2x the Infinity Cache: every weight read comes from HBM) and >= 512 MiB of outputs.
MIN_READ_FOOTPRINT = 512 << 20
MIN_WRITE_FOOTPRINT = 512 << 20
C5_MIN_STEPS = 100  # the c5 object's timed steps at least (its launches are 27-215 us)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c2", choices=["c2", "c5"])
    ap.add_argument("--m", type=int, default=None, help="override the c2 matrix shape (rows)")
    ap.add_argument("--n", type=int, default=None, help="override the c2 matrix shape (columns)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16"])
    ap.add_argument("--sets", type=int, default=0, help="rotating input AND output sets (0 = the rule below)")
    ap.add_argument("--in-sets", type=int, default=0,
                    help="rotating input sets (0 = enough for >= 512 MiB of distinct reads per rank)")
    ap.add_argument("--out-sets", type=int, default=0,
                    help="rotating output sets (0 = enough for >= 512 MiB of distinct writes per rank)")
    ap.add_argument("--repeats", type=int, default=7,
                    help="timed regions of K steps each (the median region is the result, SURVEY 8d)")
    ap.add_argument("--no-ceiling", action="store_true",
                    help="skip the memory-system twin (roofline.twin)")
    ap.add_argument("--launch", default="eager", choices=["eager", "graph"],
                    help="timed steps as eager C-ABI launches (default) or one hipGraph replay")
    ap.add_argument("--no-graph", action="store_true", help="same as --launch eager (kept for old scripts)")
    ap.add_argument("--spin-us-per-launch", type=float, default=30.0,
                    help="--lead spin-steps: device spin per launch to be submitted (us); profilers that "
                         "intercept every dispatch need more (tools/session.sh rocprof uses 150)")
    ap.add_argument("--lead", default="auto", choices=["auto", "replay", "spin", "steps", "spin-steps", "none"],
                    help="device work enqueued just ahead of the start event: an untimed graph replay, a spin "
                         "kernel, (eager) untimed launches of the preceding buffer sets, or a spin long enough "
                         "to cover the host's submission of every step followed by those launches; auto = "
                         "spin-steps for eager, none for graph")
    ap.add_argument("--lead-n", type=int, default=16, help="untimed launches just ahead of the start event (<= sets)")
    ap.add_argument("--flush", action="store_true", help="512 MiB Infinity-Cache flush before timing (A/B only)")
    ap.add_argument("--tile-dwords", type=int, default=4)
    ap.add_argument("--blocks-per-cu", type=int, default=0)
    ap.add_argument("--nontemporal", type=int, default=1)
    ap.add_argument("--flags", type=lambda v: int(v, 0), default=0,
                    help="nf4_launch_cfg.flags: reserved, must be 0 (the library rejects anything else)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="hip", choices=["hip", "cpu"])
    ap.add_argument("--no-c5", action="store_true", help="skip the BASELINE configs[4] section of the result line")
    ap.add_argument("--c5-shape", default="8192x8192", type=lambda v: tuple(int(x) for x in v.split("x")),
                    help="matrix shape of the c5 section (CPU rehearsals use a small one)")
    ap.add_argument("--dist-backend", default=None, help="nccl (= RCCL, default on GPUs) or gloo (rehearsal)")
    return ap.parse_args(argv)


_SPIN_CYCLES_PER_US = [0.0]


def _spin_rate_calibrate():
    """Cycles of torch.cuda._sleep per microsecond on this device (one timed spin)."""
    import torch

    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 2_000_000
    e0.record()
    torch.cuda._sleep(n)
    e1.record()
    torch.cuda.synchronize()
    _SPIN_CYCLES_PER_US[0] = n / max(e0.elapsed_time(e1) * 1e3, 1.0)


def spin_cycles(us: float) -> int:
    us = min(us, 50_000.0)
    return int(us * (_SPIN_CYCLES_PER_US[0] or 100.0))


# ---------------------------------------------------------------------------
# launcher: N fresh rank processes (no GPU call in this process)
# ---------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """Run this script as N ranks (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*), relay their
    output, return the worst exit code.  The parent never initialises the GPU, so
    the children are plain fresh processes (no exec from a GPU-initialised one)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # poll every rank: the first one to fail ends the others (they would otherwise sit
    # in init_process_group or a barrier until the backend's timeout)
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            log(f"bench.py: a rank exited with {bad[0]}; the other ranks were stopped")
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.05)


# ---------------------------------------------------------------------------
# workload
# ---------------------------------------------------------------------------
def rank_matrices(args, rank: int, world: int):
    """[(global matrix id, m, n)] this rank dequantizes per step."""
    if args.workload == "c5":
        import workloads as W

        m, n = W.C5_SHAPE
        return [(i, m, n) for i in range(rank, W.C5_MATRICES, world)]
    m = args.m or 4096
    n = args.n or 4096
    return [(rank, m, n)]


def algorithmic_bytes(m, n, out_bytes, nb, n2):
    import workloads as W

    return W.algorithmic_bytes(m, n, out_bytes, nb, n2)


def cpu_baseline(shapes, seconds, dtype_code):
    """CPU figures on the same workload (the rank's step), on this GPU's host share
    of cores (<= 16): the reference fallback's structure in torch-CPU (``value``),
    this library's host path (``native``) and the same at one thread."""
    import torch

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import fallback_torch as F  # the baseline's reference-structure port (checker side)
    import workloads as W
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1))
    m, n = shapes[0][1], shapes[0][2]
    p, a1, a2 = W.make_inputs(m, n, 3409)
    elems = m * n

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

    tdt = torch.bfloat16 if dtype_code == _lib.BF16 else torch.float16
    tp, ta1, ta2 = torch.from_numpy(p), torch.from_numpy(a1), torch.from_numpy(a2)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        rf, ef = repeat(lambda: F.dequant_fallback(tp, ta1, ta2, m, n, tdt), seconds)
    finally:
        torch.set_num_threads(prev)
    out = np.empty((m, n), np.uint16)

    def native(nthreads, secs):
        def once():
            rc = L.nf4_dequant_ref_cpu(p.ctypes.data, p.size, a1.ctypes.data, a1.size, a2.ctypes.data, a2.size,
                                       out.ctypes.data, dtype_code, m, n, nthreads)
            if rc:
                raise RuntimeError(f"nf4_dequant_ref_cpu: {_lib.strerror(rc)}")
        return repeat(once, secs)

    rn, en = native(threads, max(1.0, seconds / 4))
    r1, e1 = native(1, max(1.0, seconds / 4))
    dname = "bf16" if dtype_code == _lib.BF16 else "fp16"
    return {"value": rf * elems / ef, "unit": "elements/s", "cores": threads, "kind": "port",
            "sample": f"{rf} x {m}x{n} NF4->{dname} by oracle/fallback_torch.py (the reference fallback's "
                      f"loop structure in torch-CPU, bit-equal to it, {threads} threads), {ef:.1f} s",
            "native": {"value": rn * elems / en, "cores": threads,
                       "sample": f"{rn} x {m}x{n} by libnf4dq.so nf4_dequant_ref_cpu (this library's host path, "
                                 f"AVX2 table lookups, {threads} threads), {en:.1f} s"},
            "single_thread": {"value": r1 * elems / e1, "cores": 1,
                              "sample": f"{r1} x {m}x{n} by nf4_dequant_ref_cpu, 1 thread, {e1:.1f} s"}}


def find_traffic(m, n, dtype):
    for rnd, name in [(r, f) for r in ROUNDS for f in ("pmc_traffic.json", f"pmc_traffic_{dtype}.json")]:
        path = os.path.join(REPO, "profiles", rnd, name)
        if not os.path.exists(path):
            continue
        try:
            with open(path) as f:
                pmc = json.load(f)
        except (OSError, ValueError):
            continue
        if pmc.get("m") == m and pmc.get("n") == n and pmc.get("dtype") == dtype:
            return pmc.get("hbm_bytes_per_launch"), f"profiles/{rnd}/{name}"
    return None, None


def step_bytes(mats):
    """(distinct bytes one step reads, bytes it writes) for a rank's matrices."""
    rd = sum(m * n // 2 + m * n // 64 + 4 * ((m * n // 64 + 255) // 256) for _, m, n in mats)
    return rd, sum(2 * m * n for _, m, n in mats)


def rotation_sets(mats):
    """(input sets, output sets) of the HBM-streamed rotation: >= 512 MiB of distinct
    reads and >= 512 MiB of distinct writes per rank, at every N."""
    rd, wr = step_bytes(mats)
    return max(1, -(-MIN_READ_FOOTPRINT // max(1, rd))), max(1, -(-MIN_WRITE_FOOTPRINT // max(1, wr)))


class Workload:
    """One rank's share of a workload: its matrices, Pin rotating input sets (packed
    weight + this rank's scattered quant statistics) and Pout rotating output sets on
    the device, and one bound C-ABI call per (input set, output set) pair used (step i
    reads input i % Pin and writes output i % Pout; arguments prepared up front)."""

    def __init__(self, args, mats, stats, dev, dt, code, cfg_p, cpu, pin=0, pout=0):
        import torch

        import workloads as W
        from nf4_triton_dequantization_amd import _lib

        self.mats, self.cpu, self.code, self.cfg_p = mats, cpu, code, cfg_p
        self.L = _lib.lib()
        self._lib = _lib
        read_step, write_step = step_bytes(mats)
        if cpu:
            pin = pin or args.sets or 2
            pout = pout or args.sets or 2
        else:
            rin, rout = rotation_sets(mats)
            pin = pin or args.in_sets or args.sets or rin
            pout = pout or args.out_sets or args.sets or rout
            if not (args.sets or args.in_sets) and args.launch == "graph" and not args.no_graph:
                # graph replay: across the boundary between two replays input set 0 recurs
                # after K - Pin*floor((K-1)/Pin) steps (K when Pin >= K): keep the reads in
                # between >= 512 MiB so no weight is still in the Infinity Cache when reached
                def reuse(p):
                    return args.steps if p >= args.steps else args.steps - p * ((args.steps - 1) // p)

                while pin < args.steps and reuse(pin) * read_step < MIN_READ_FOOTPRINT:
                    pin += 1
        self.Pin, self.Pout = pin, pout
        self.P = max(pin, pout)  # one pass over every input and output set
        self.read_bytes, self.write_bytes = pin * read_step, pout * write_step
        # one host generation per matrix; the sets are device copies (distinct
        # addresses are what keep a set out of the caches, not distinct contents)
        base = []
        for (gid, m, n), st in zip(mats, stats):
            q = torch.from_numpy(W.splitmix64_bytes(3409 + 7919 * gid, m * n // 2, stream=1)).to(dev)
            base.append((q, st.absmax.to(dev), st.absmax2.to(dev), m, n))
        self.ins = []
        for s_i in range(pin):
            row = []
            for (q, a1, a2, m, n) in base:
                if s_i:
                    q, a1, a2 = q.clone(), a1.clone(), a2.clone()
                row.append((q, a1, a2, m, n))
            self.ins.append(row)
        self.outs = [[torch.empty((m, n), dtype=dt, device=dev) for (_, m, n) in mats] for _ in range(pout)]
        self.sp = None if cpu else torch.cuda.current_stream(dev).cuda_stream
        self._calls = {}

    def _call(self, a, b):
        """The bound launch of input set a into output set b (built once)."""
        fn = self._calls.get((a, b))
        if fn is not None:
            return fn
        _lib, L = self._lib, self.L
        row, outs = self.ins[a], self.outs[b]
        if len(row) == 1:
            q, a1, a2, m, n = row[0]
            args_ = (q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                     outs[0].data_ptr(), self.code, m, n)
            f = L.nf4_dequant_ref if self.cfg_p is None else L.nf4_dequant_ref_cfg
            args_ = args_ + ((self.sp,) if self.cfg_p is None else (self.cfg_p, self.sp))
        else:
            descs = (_lib.MatrixDesc * len(row))(*[
                _lib.MatrixDesc(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                out.data_ptr(), m, n) for (q, a1, a2, m, n), out in zip(row, outs)])
            f, args_ = L.nf4_dequant_ref_batched, (descs, len(row), self.code, self.sp)

        def call(f=f, a=args_):
            rc = f(*a)
            if rc:
                raise RuntimeError(f"nf4 dequant launch: {_lib.strerror(rc)}")
        self._calls[(a, b)] = call
        return call

    def step_call(self, i):
        return self._call(i % self.Pin, i % self.Pout)

    def launch(self, i):
        if not self.cpu:
            self.step_call(i)()
            return
        _lib = self._lib
        for (q, a1, a2, m, n), out in zip(self.ins[i % self.Pin], self.outs[i % self.Pout]):
            rc = self.L.nf4_dequant_ref_cpu(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(),
                                            a2.numel(), out.data_ptr(), self.code, m, n, 0)
            if rc:
                raise RuntimeError(f"nf4_dequant_ref_cpu: {_lib.strerror(rc)}")

    def sanity(self, dtype_name):
        """Step 0's output (input set 0 -> output set 0) against the oracle on the first
        64 rows of each matrix (the checker; tests/ do the full job)."""
        import torch

        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import nf4_oracle as O

        for (q, a1, a2, m, n), out in zip(self.ins[0], self.outs[0]):
            r = min(64, m)
            want = O.dequant_ref_np(q[: r * n // 2].cpu().numpy(), a1.cpu().numpy(), a2.cpu().numpy(), r, n,
                                    O.BF16 if dtype_name == "bf16" else O.F16)
            got = out[:r].contiguous().view(torch.int16).cpu().numpy().view(np.uint16)
            if not np.array_equal(got, want):
                raise RuntimeError("bench sanity check failed: output differs from the oracle")
        return True

    def regime(self):
        """What the rotation makes of the caches (recorded in the line)."""
        return {"in_sets": self.Pin, "out_sets": self.Pout, "read_footprint_bytes": self.read_bytes,
                "write_footprint_bytes": self.write_bytes,
                "weights_from": ("HBM (distinct reads >= 512 MiB, 2x the Infinity Cache)"
                                 if self.read_bytes >= MIN_READ_FOOTPRINT else
                                 "Infinity Cache possible (distinct reads < 512 MiB)")}

    def elements(self):
        return sum(m * n for _, m, n in self.mats)

    def alg_bytes(self):
        return sum(algorithmic_bytes(m, n, 2, m * n // 64, (m * n // 64 + 255) // 256) for _, m, n in self.mats)


def time_steps(args, wl, dev, world, graph_ok=True):
    """Warmup, one untimed pass over every buffer set, then ``--repeats`` timed regions
    of exactly K steps each (see the module docstring), every region bracketed by a
    barrier + synchronize on both sides; returns ([ms for K steps on this rank, one per
    region], launch mode)."""
    import torch
    import torch.distributed as dist

    cpu = wl.cpu
    P = wl.P
    lead_n = min(args.lead_n, P)
    for w in range(args.warmup):
        wl.launch(w)
    if not cpu:
        # one untimed pass over every input and output set: the first touch of a set's
        # pages costs +1.5-3 us per 42 MB launch in GPU TLB misses (profiles/r02/bench_lead_ab.txt,
        # profiles/r02/bench_eager_ab.txt) -- the steady state of a resident weight
        # set is TLB-warm; the graph path's untimed replay did this implicitly
        for s_i in range(P):
            wl.step_call(s_i)()
        torch.cuda.synchronize()
    graph = None
    if graph_ok and not cpu and args.launch == "graph" and not args.no_graph:
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for i in range(args.steps):
                    wl.launch(i)
            graph.replay()  # upload + one untimed pass
            torch.cuda.synchronize()
        except Exception as e:  # capture unsupported -> eager issue, reported in config
            log(f"hipGraph capture failed ({e}); timing eager launches")
            graph = None
            torch.cuda.synchronize()
    if not cpu and args.flush:
        # optional: evict the Infinity Cache with a 512 MiB scratch write (measured:
        # costs 1-2 us per step afterwards -- the new allocation's mappings evict the
        # GPU TLBs -- so the buffer-set rule above is the default hygiene instead)
        scratch = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
        scratch.fill_(1)
        torch.cuda.synchronize()
        del scratch
    if not cpu and args.lead == "spin-steps":
        _spin_rate_calibrate()
    times = []
    calls = [wl.step_call(i) for i in range(args.steps)] if not cpu else None  # bound before anything is timed
    if not cpu:
        main_stream = torch.cuda.current_stream(dev)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
    for _rep in range(max(1, args.repeats)):
        if world > 1:
            dist.barrier()
        if not cpu:
            torch.cuda.synchronize()
        if cpu:
            t0 = time.perf_counter()
            for i in range(args.steps):
                wl.launch(i)
            times.append((time.perf_counter() - t0) * 1e3)
        else:
            if graph is not None and args.lead == "replay":
                # one more untimed replay enqueued right ahead of the start event: the
                # timed steps follow warm steps back to back (as in a steady stream of
                # work) and the host's submission of the timed replay hides behind it
                graph.replay()
            elif args.lead == "spin":
                torch.cuda._sleep(100_000)  # device spin: hides only the host's submission
            elif graph is None and args.lead == "spin-steps":
                # a device spin that outlasts the host's submission of every launch below
                # (a profiler's per-dispatch interception makes submission ~10 us per launch,
                # slower than the kernels: without the spin the timed launches would trickle
                # in one by one), then the untimed launches of the preceding sets
                torch.cuda._sleep(spin_cycles(args.spin_us_per_launch * (args.steps + lead_n) + 200.0))
                for j in range(lead_n):
                    wl.step_call(j - lead_n)()
            elif graph is None and args.lead == "steps":
                # untimed launches of the sets just before the timed ones (steps -L..-1):
                # the queue holds real work when the start event fires, as in a steady
                # stream of weights, so host launch latency never idles the GPU
                for j in range(lead_n):
                    wl.step_call(j - lead_n)()
            ev0.record(main_stream)
            if graph is not None:
                graph.replay()
            else:
                for c in calls:
                    c()
            ev1.record(main_stream)
            torch.cuda.synchronize()
            times.append(ev0.elapsed_time(ev1))
        if world > 1:
            dist.barrier()
    mode = "hipGraph" if graph is not None else ("host loop" if cpu else "eager")
    return times, mode


def median_region(my_times, dev, world):
    """The result of R timed regions: per region the max over ranks (the slowest rank
    decides), then the region with the median of those maxima.  Returns (its time,
    every rank's time in that region, the per-region maxima in region order)."""
    R = len(my_times)
    if world == 1:
        maxima, table = list(my_times), [list(my_times)]
    else:
        import torch.distributed as dist

        from nf4_triton_dequantization_amd.sharding import max_over_ranks

        maxima = [max_over_ranks(t, dev) for t in my_times]
        table = [None] * world
        dist.all_gather_object(table, list(my_times))
    order = sorted(range(R), key=lambda i: maxima[i])
    pick = order[(R - 1) // 2]  # the lower median for even R: always one measured region
    return maxima[pick], [table[r][pick] for r in range(world)], maxima


class TwinWorkload:
    """The memory-system twin of a one-matrix step (tools/stream_probe.hip ``twin_mix``):
    the flat kernel's packed-weight loads (4 B/lane, nt) and output stores (16 B/lane,
    sc1 + nt) over the same tile grid, no decode and no scale loads, on the same
    rotation rule (>= 512 MiB of distinct reads, >= 512 MiB of distinct writes)."""

    cpu = False

    def __init__(self, lib, m, n, dev):
        import torch

        self.L, self.nbytes = lib, m * n // 2
        pin, pout = rotation_sets([(0, m, n)])
        self.Pin, self.Pout, self.P = pin, pout, max(pin, pout)
        self.ins = [torch.randint(0, 256, (self.nbytes,), dtype=torch.uint8, device=dev) for _ in range(pin)]
        self.outs = [torch.empty((m, n), dtype=torch.bfloat16, device=dev) for _ in range(pout)]
        self.sink = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
        self.sp = torch.cuda.current_stream(dev).cuda_stream

    def step_call(self, i):
        a, b = self.ins[i % self.Pin].data_ptr(), self.outs[i % self.Pout].data_ptr()

        def call(L=self.L, a=a, b=b):
            rc = L.twin_launch(0, 2, 18, 1, a, self.nbytes, b, self.sink.data_ptr(), self.sp)
            if rc:
                raise RuntimeError(f"twin_launch: {rc}")
        return call

    def launch(self, i):
        self.step_call(i)()


def twin_measure(args, mat, dev, world, rank, alg, kernel_us):
    """Time the memory-system twin of this rank's step exactly as the headline (same K,
    repeats, lead, spin): a reference point for the access pattern, not a bound (the
    product beats it)."""
    import torch

    path = os.path.join(REPO, "tools", "_build", "libstreamprobe.so")
    if not os.path.exists(path):
        log("bench.py: tools/_build/libstreamprobe.so missing; no twin")
        return None
    _, m, n = mat
    if m * n // 2 >= 1 << 30:  # the twin's output range is nbytes * 4 in 32 bits (stream_probe.hip)
        log("bench.py: matrix past the twin's 32-bit output range; no twin")
        return None
    L = ctypes.CDLL(path)
    L.twin_launch.restype = ctypes.c_int
    L.twin_launch.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_void_p]
    tw = TwinWorkload(L, m, n, dev)
    times, _ = time_steps(args, tw, dev, world, graph_ok=False)
    _, per, _ = median_region(times, dev, world)
    us = per[rank] * 1e3 / args.steps
    del tw
    torch.cuda.empty_cache()
    return {"kernel": "twin_mix (tools/stream_probe.hip): the flat kernel's loads and stores, no decode",
            "launch_us": us, "achieved": alg / (us * 1e-6) / 1e9, "frac": alg / (us * 1e-6) / PEAK_HBM,
            "kernel_over_twin": kernel_us / us,
            "method": "same rotation, K, repeats, lead and spin as the headline, timed right after it",
            "note": ("a reference point, not a ceiling: the twin has the product's one-tile loads and "
                     "stores but no scale gathers and no decode, and the product is faster than it "
                     "(kernel_over_twin < 1, DESIGN.md section 4)")}


def distribute_stats(all_mats, rank, world, dev, dt, cpu):
    """Rank 0 holds every matrix's quant statistics (as after loading a checkpoint);
    each rank receives only its own matrices' (sharding.scatter_quant_stats over
    RCCL).  Returns (this rank's stats, ms the distribution took)."""
    import torch

    import workloads as W
    from nf4_triton_dequantization_amd.sharding import QuantStats, scatter_quant_stats

    def sync():
        if not cpu:
            torch.cuda.synchronize()

    per_rank = None
    if rank == 0:
        per_rank = []
        for r in range(world):
            row = []
            for gid, m, n in all_mats[r]:
                seed = 3409 + 7919 * gid
                nb = m * n // 64
                row.append(QuantStats(m, n, torch.from_numpy(W.splitmix64_bytes(seed, nb, stream=2)),
                                      torch.from_numpy(W.uniform_f32(seed, (nb + 255) // 256, 1e-3, 1e-2,
                                                                     stream=3)), dt))
            per_rank.append(row)
    import torch.distributed as dist

    if not dist.is_initialized():
        return [QuantStats(s.m, s.n, s.absmax.to(dev), s.absmax2.to(dev), s.dtype) for s in per_rank[0]], 0.0

    dist.barrier()
    sync()
    tb = time.perf_counter()
    mine = scatter_quant_stats(per_rank, dev, src=0)
    sync()
    return mine, (time.perf_counter() - tb) * 1e3


def rank_figures(all_mats, per_rank_ms, steps):
    out = []
    for r, ms in enumerate(per_rank_ms):
        el = sum(m * n for _, m, n in all_mats[r])
        by = sum(algorithmic_bytes(m, n, 2, m * n // 64, (m * n // 64 + 255) // 256) for _, m, n in all_mats[r])
        out.append({"rank": r, "matrices": len(all_mats[r]), "ms_per_step": ms / steps,
                    "elements_per_s": el * steps / (ms * 1e-3), "GBps": by * steps / (ms * 1e-3) / 1e9})
    return out


def c5_section(args, rank, world, dev, dt, code, cpu):
    """BASELINE configs[4] at this N: the 8 independent c5 matrices split round-robin
    over the ranks (one per GPU at N = 8), each rank's share one launch per step
    (the single-matrix entry at N = 8, the batched one below), quant statistics
    scattered from rank 0.  Aggregate = 8 matrices / the slowest rank's time."""
    import copy

    import torch

    import workloads as W

    # timed over max(K, C5_MIN_STEPS) steps: at the driver's K = 20 the first launches
    # after the lead weigh 1-2 % of a 20-step region (78.5 % at K = 200 vs 76.7 % at
    # K = 20 on one box, profiles/r04/final/); the headline keeps exactly K
    args = copy.copy(args)
    args.steps = max(args.steps, C5_MIN_STEPS)
    m, n = args.c5_shape
    all_mats = [[(g, m, n) for g in range(r, W.C5_MATRICES, world)] for r in range(world)]
    mats = all_mats[rank]
    stats, scatter_ms = distribute_stats(all_mats, rank, world, dev, dt, cpu)
    wl = Workload(args, mats, stats, dev, dt, code, None, cpu)
    wl.launch(0)
    if not cpu:
        torch.cuda.synchronize()
    verified = wl.sanity(args.dtype) if mats else True
    my_times, _mode = time_steps(args, wl, dev, world, graph_ok=False)
    t_ms, per, _maxima = median_region(my_times, dev, world)
    els = W.C5_MATRICES * m * n
    alg = W.C5_MATRICES * algorithmic_bytes(m, n, 2, m * n // 64, (m * n // 64 + 255) // 256)
    per_rank = rank_figures(all_mats, per, args.steps)
    gbps = alg * args.steps / (t_ms * 1e-3) / 1e9
    res = {
        "config": f"c5: {W.C5_MATRICES} independent {m}x{n} NF4->{args.dtype} matrices (BASELINE configs[4]) "
                  f"split round-robin over {world} rank(s)",
        "matrices": W.C5_MATRICES, "shape": [m, n], "n_gpus": world, "steps": args.steps,
        "ms_per_step": t_ms / args.steps, "elements_per_s": els * args.steps / (t_ms * 1e-3), "GBps": gbps,
        "frac_of_peak": None if cpu else gbps * 1e9 / (PEAK_HBM * world),
        "per_rank": per_rank, "scaling": "strong",
        "launch": ("one nf4_dequant_ref launch per rank per step" if max(len(a) for a in all_mats) == 1 else
                   "each rank's share in one nf4_dequant_ref_batched launch per step"),
        "buffer_sets": wl.P, "regime": wl.regime(), "quant_state_scatter_ms": round(scatter_ms, 3),
        "quant_state_bytes_per_rank": [sum(m * n // 64 + 4 * ((m * n // 64 + 255) // 256) for _ in a)
                                       for a in all_mats],
        "verified_first_rows": bool(verified),
    }
    del wl
    if not cpu:
        torch.cuda.empty_cache()
    return res


def c5_cpu_figures(args, code, threads):
    """Host-CPU figures for one c5 matrix on rank 0: this library's host path (native)
    and the reference-structure torch port, one matrix each (bounded sample)."""
    import torch

    import workloads as W
    from nf4_triton_dequantization_amd import _lib

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import fallback_torch as F

    m, n = args.c5_shape
    p, a1, a2 = W.make_inputs(m, n, 3409)
    out = np.empty((m, n), np.uint16)
    L = _lib.lib()
    t0 = time.perf_counter()
    reps = 0
    while reps < 3 or time.perf_counter() - t0 < 1.0:
        rc = L.nf4_dequant_ref_cpu(p.ctypes.data, p.size, a1.ctypes.data, a1.size, a2.ctypes.data, a2.size,
                                   out.ctypes.data, code, m, n, threads)
        if rc:
            raise RuntimeError(f"nf4_dequant_ref_cpu: {_lib.strerror(rc)}")
        reps += 1
    native = reps * m * n / (time.perf_counter() - t0)
    tdt = torch.bfloat16 if code == _lib.BF16 else torch.float16
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        t0 = time.perf_counter()
        F.dequant_fallback(torch.from_numpy(p), torch.from_numpy(a1), torch.from_numpy(a2), m, n, tdt)
        port = m * n / (time.perf_counter() - t0)
    finally:
        torch.set_num_threads(prev)
    return {"unit": "elements/s", "cores": threads, "kind": "port", "value": port, "native": native,
            "sample": f"one {m}x{n} matrix: oracle/fallback_torch.py once, nf4_dequant_ref_cpu x{reps}"}


def main():
    args = parse_args()
    if args.lead == "auto":
        args.lead = "none" if args.launch == "graph" and not args.no_graph else "spin-steps"
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(world_env or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; they must agree")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("NF4_BENCH_FAIL_RANK") == str(rank):  # test hook: a rank that dies at startup
        raise SystemExit(f"bench.py: rank {rank} failing on request (NF4_BENCH_FAIL_RANK)")
    # stdout carries exactly one line, the result: anything the runtime libraries
    # print there (gloo's connection notes, RCCL / HIP warnings) goes to stderr
    result_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    from nf4_triton_dequantization_amd import _lib

    cpu = args.backend == "cpu"
    dist_backend = args.dist_backend or ("gloo" if cpu else "nccl")
    if cpu:
        dev = torch.device("cpu")
    else:
        # rehearsal with more ranks than GPUs (gloo only): ranks share devices
        ndev = torch.cuda.device_count()
        if dist_backend == "nccl" and (local >= ndev or world > ndev):
            # one rank per GPU over RCCL: more ranks than visible devices cannot form the
            # group (set_device would fail, or two ranks would share a GPU); say so plainly
            raise SystemExit(f"bench.py: --dist-backend nccl needs one GPU per rank: WORLD_SIZE={world}, "
                             f"LOCAL_RANK={local}, but this node shows {ndev} GPU(s) "
                             f"(use --dist-backend gloo to rehearse more ranks)")
        local_dev = local if dist_backend == "nccl" else local % max(1, ndev)
        torch.cuda.set_device(local_dev)
        dev = torch.device("cuda", local_dev)
    if world > 1 or args.dist_backend:
        # an explicit --dist-backend at N = 1 still forms the (one-rank) group, so the
        # RCCL scatter of the quant statistics runs on one GPU too
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(dist_backend)

    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    code = _lib.BF16 if args.dtype == "bf16" else _lib.F16
    cfg = _lib.LaunchCfg(args.tile_dwords, args.blocks_per_cu, args.nontemporal, args.flags)
    default_cfg = (args.tile_dwords, args.blocks_per_cu, args.nontemporal, args.flags) == (4, 0, 1, 0)
    cfg_p = None if default_cfg else ctypes.byref(cfg)

    # ---- headline workload: setup (quant statistics scattered from rank 0) ----------------
    all_mats = [rank_matrices(args, r, world) for r in range(world)]
    mats = all_mats[rank]
    t_setup = time.perf_counter()
    stats, scatter_ms = distribute_stats(all_mats, rank, world, dev, dt, cpu)
    wl = Workload(args, mats, stats, dev, dt, code, cfg_p, cpu)
    if not cpu:
        torch.cuda.synchronize()
    log(f"[rank {rank}] setup {time.perf_counter() - t_setup:.1f}s, {wl.Pin} input / {wl.Pout} output sets x "
        f"{len(mats)} matrices, quant_state scatter {scatter_ms:.2f} ms")
    wl.launch(0)
    if not cpu:
        torch.cuda.synchronize()
    wl.sanity(args.dtype)

    # ---- timed regions: R repeats of exactly K steps, the median region is the result ---------
    my_times, launch_mode = time_steps(args, wl, dev, world)
    t_ms, per_rank_ms, maxima = median_region(my_times, dev, world)

    # ---- figures -------------------------------------------------------------------------------
    my_alg = wl.alg_bytes()
    launches_per_step = 1 if not cpu else len(mats)
    all_elems = sum(m * n for r in range(world) for _, m, n in all_mats[r])
    all_alg = sum(algorithmic_bytes(m, n, 2, m * n // 64, (m * n // 64 + 255) // 256)
                  for r in range(world) for _, m, n in all_mats[r])
    value = all_elems * args.steps / (t_ms * 1e-3)
    my_ms = per_rank_ms[rank]  # this rank's time in the median region
    kt = my_ms * 1e3 / (args.steps * launches_per_step)  # us per launch, this rank
    kts = sorted(t * 1e3 / (args.steps * launches_per_step) for t in my_times)
    m0, n0 = mats[0][1], mats[0][2]
    traffic, traffic_src = (None, None)
    if not cpu and len(mats) == 1:
        traffic, traffic_src = find_traffic(m0, n0, args.dtype)
    achieved = my_alg / launches_per_step / (kt * 1e-6)
    regime = wl.regime()
    del wl
    if not cpu:
        torch.cuda.empty_cache()
    # ---- the memory-system twin (reported, never `value`): the same loads and stores
    # with no decode, timed the same way on the same rotation -- a reference point for
    # the access pattern, not a ceiling (tools/stream_probe.hip twin_mix) ----------------------
    twin = None
    if not cpu and not args.no_ceiling and len(mats) == 1 and args.launch == "eager":
        twin = twin_measure(args, mats[0], dev, world, rank, my_alg, kt)
    if args.workload == "c5":
        metric = "dequantized elements/s (8 x 8192x8192 NF4->bf16, one matrix per GPU at N=8)"
        workload = (f"c5: 8 independent 8192x8192 NF4->{args.dtype} matrices (BASELINE configs[4]) split "
                    f"round-robin over {world} rank(s), each rank's share in one batched launch per step")
        scaling = "strong"
    else:
        metric = "dequantized elements/s (4096x4096 NF4->bf16, blocksize 64 / nested 256)"
        workload = (f"c2: {m0}x{n0} NF4->{args.dtype} double dequant (BASELINE configs[1]), one matrix per rank "
                    f"per step")
        scaling = "weak"
    res = {
        "metric": metric,
        "value": value,
        "unit": "elements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_ms / args.steps,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (splitmix64 packed weights + absmax, resident in HBM)",
        "hbm_gb_s": all_alg * args.steps / (t_ms * 1e-3) / 1e9,
        "per_rank": rank_figures(all_mats, per_rank_ms, args.steps),
        "config": {
            "workload": workload,
            "matrices_per_rank": len(mats), "m": m0, "n": n0, "out_dtype": args.dtype,
            "arith": "u8 unpack, fp32 scale/multiply, RNE to bf16/fp16", "backend": args.backend,
            "buffer_sets": args.sets or None, "launch": launch_mode, "rotation": regime,
            "tile_dwords": args.tile_dwords, "blocks_per_cu": args.blocks_per_cu, "nontemporal": args.nontemporal,
            "flags": args.flags, "parallelism": f"shard{world} (independent matrices)",
            "cache_flush_before_timing": bool(not cpu and args.flush), "lead": args.lead,
            "quant_state_scatter_ms": round(scatter_ms, 3), "dist_backend": dist_backend if dist.is_initialized() else None,
        },
        "roofline": None if cpu else {
            "bound": "hbm",
            "achieved": achieved / 1e9,
            "peak": PEAK_HBM / 1e9,
            "unit": "GB/s",
            "frac": achieved / PEAK_HBM,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": "nf4_flat_kernel",
            "launch_us": kt,
            "launch_us_min": kts[0],
            "launch_us_median": kts[(len(kts) - 1) // 2],
            "launch_us_max": kts[-1],
            "launch_us_source": (f"HIP events on the launch stream over each of {len(my_times)} timed regions of "
                                 f"{args.steps} steps (gaps included) / launches; the region with the median "
                                 f"max-over-ranks time is the result"),
            "algorithmic_bytes_per_launch": my_alg // launches_per_step,
            "twin": twin,
            "measured_copy_peak": MEASURED_COPY / 1e9,
            "frac_of_measured_copy": achieved / MEASURED_COPY,
            "measured_copy_source": "MI355X_MICROARCH.md: HBM3E 6.29 TB/s measured (float4 copy)",
        },
        "repeats": {"regions": len(maxima), "steps_per_region": args.steps,
                    "ms_per_step_by_region": [t / args.steps for t in maxima]},
        "cpu_baseline": None,
        "c5": None,
    }
    # ---- BASELINE configs[4] at this N (every N: the driver's scaling runs carry it) --------
    if not args.no_c5 and args.workload != "c5":
        res["c5"] = c5_section(args, rank, world, dev, dt, code, cpu)
    # ---- CPU baseline: rank 0, after every timed region, at every N ---------------------------
    if rank == 0 and not args.no_cpu_baseline:
        threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1))
        res["cpu_baseline"] = cpu_baseline(mats, args.cpu_seconds, code)
        if res["c5"] is not None:
            res["c5"]["cpu_baseline"] = c5_cpu_figures(args, code, threads)
    if rank == 0:
        print(json.dumps(res), file=result_out, flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
