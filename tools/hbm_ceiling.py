"""What the memory system gives the dequant's access mix (speed-of-light check).

Times, with hipGraph replay over inputs and outputs rotated independently (>= 512
MiB of distinct reads: the weights stream from HBM, profiles/r04/cache/):
  * calib_mix  -- nf4_flat_kernel's exact load/store shapes, no decode
                  (1 B read : 4 B written, like NF4 -> 16-bit)
  * calib_mix16 -- 16 B/lane loads (1 KiB per wave instruction), four strided 16 B
                  stores per lane (the alternative tile shape)
  * nf4 dequant (bench default config) on the same sizes
  * calib_read / calib_write on 1 GiB (pure streams)
Prints JSON lines: GB/s and fraction of the 8 TB/s spec.
"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from nf4_triton_dequantization_amd import _lib  # noqa: E402

PEAK = 8e12


def graph_time(fn, steps, reps=5):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(steps):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    st = torch.cuda.current_stream()
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3 / steps)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda", 0)
    C = ctypes.CDLL(os.path.join(REPO, "tools", "_build", "libpmccalib.so"))
    L = _lib.lib()
    for (m, n) in ((4096, 4096), (8192, 8192)):
        # round 4: inputs and outputs rotate independently, >= 512 MiB of distinct reads
        # (the weights stream from HBM, as in bench.py) and >= 512 MiB of outputs
        nbytes = m * n // 2
        nb = m * n // 64
        PI = -(-(512 << 20) // nbytes)
        PO = -(-(512 << 20) // (4 * nbytes))
        ins = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev) for _ in range(PI)]
        outs = [torch.empty((m, n), dtype=torch.bfloat16, device=dev) for _ in range(PO)]
        a1 = torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev)
        a2 = torch.rand((nb + 255) // 256, device=dev)

        def mix(i):
            assert C.calib_mix_launch(ctypes.c_void_p(ins[i % PI].data_ptr()), ctypes.c_uint32(nbytes),
                                      ctypes.c_void_p(outs[i % PO].data_ptr()),
                                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0

        def mix16(i):
            assert C.calib_mix16_launch(ctypes.c_void_p(ins[i % PI].data_ptr()), ctypes.c_uint32(nbytes),
                                        ctypes.c_void_p(outs[i % PO].data_ptr()),
                                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0

        def deq(i):
            assert L.nf4_dequant_ref(ins[i % PI].data_ptr(), nbytes, a1.data_ptr(), nb, a2.data_ptr(), a2.numel(),
                                     outs[i % PO].data_ptr(), _lib.BF16, m, n,
                                     torch.cuda.current_stream().cuda_stream) == 0

        for name, fn, byt in (("calib_mix (same access shapes and policies, no decode)", mix, nbytes * 5),
                              ("calib_mix16 (16 B/lane loads, strided 16 B stores)", mix16, nbytes * 5),
                              ("nf4 dequant", deq, nbytes * 5 + nb + 4 * a2.numel())):
            t = graph_time(fn, 2 * PI)
            print(json.dumps({"kernel": name, "m": m, "n": n, "in_sets": PI, "out_sets": PO, "us": t * 1e6,
                              "GBps": byt / t / 1e9, "frac": byt / t / PEAK}), flush=True)
        del ins, outs
        torch.cuda.empty_cache()
    buf = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    sink = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    t = graph_time(lambda i: C.calib_read(ctypes.c_void_p(buf.data_ptr()), ctypes.c_uint32(1 << 30),
                                          ctypes.c_void_p(sink.data_ptr()), st()), 8)
    print(json.dumps({"kernel": "calib_read 1 GiB (4 B/lane loads)", "us": t * 1e6, "GBps": (1 << 30) / t / 1e9,
                      "frac": (1 << 30) / t / PEAK}))
    t = graph_time(lambda i: C.calib_write(ctypes.c_void_p(buf.data_ptr()), ctypes.c_uint32(1 << 30), st()), 8)
    print(json.dumps({"kernel": "calib_write 1 GiB (16 B/lane nt stores)", "us": t * 1e6,
                      "GBps": (1 << 30) / t / 1e9, "frac": (1 << 30) / t / PEAK}))


if __name__ == "__main__":
    main()
