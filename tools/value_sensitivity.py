"""Diagnostics: does the placement of the small absmax arrays change the dequant time?

Compares, in one process (interleaved rounds), 4096^2 and 8192^2 NF4->bf16 over
rotating packed/output buffers with (a) one shared absmax/nested-absmax pair and
(b) a separate pair per buffer set (what bench.py does), (c) per-set absmax bytes
as slices of one large allocation.
"""
import ctypes, json, os, sys  # noqa: E401

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tools")]
from nf4_triton_dequantization_amd import _lib  # noqa: E402
from hbm_ceiling import graph_time  # noqa: E402

L = _lib.lib()
dev = torch.device("cuda", 0)
for (m, n, P) in ((4096, 4096, 16), (8192, 8192, 8)):
    nbytes, nb = m * n // 2, m * n // 64
    n2 = (nb + 255) // 256
    ins = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev) for _ in range(P)]
    outs = [torch.empty((m, n), dtype=torch.bfloat16, device=dev) for _ in range(P)]
    a1s = [torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev) for _ in range(P)]
    a2s = [torch.rand(n2, device=dev) * 0.01 + 1e-3 for _ in range(P)]
    # the same per-set bytes as views into one large allocation (2 MiB-aligned slices):
    # separates "different bytes per set" from "separate small-pool allocations"
    slab = torch.empty(P * (2 << 20), dtype=torch.uint8, device=dev)
    a1v = [slab[i * (2 << 20): i * (2 << 20) + nb] for i in range(P)]
    for i in range(P):
        a1v[i].copy_(a1s[i])
    print(json.dumps({"m": m, "a1_alloc": [int(t.data_ptr()) % (2 << 20) for t in a1s[:4]],
                      "slab_mod_2MiB": int(slab.data_ptr()) % (2 << 20)}), flush=True)
    variants = {"shared a1/a2": lambda i: (a1s[0], a2s[0]), "per-set a1/a2": lambda i: (a1s[i % P], a2s[i % P]),
                "per-set a1, shared a2": lambda i: (a1s[i % P], a2s[0]),
                "shared a1, per-set a2": lambda i: (a1s[0], a2s[i % P]),
                "per-set a1 in one slab, shared a2": lambda i: (a1v[i % P], a2s[0])}
    for r in range(3):
        for name, pick in variants.items():
            def deq(i, pick=pick):
                a1, a2 = pick(i)
                assert L.nf4_dequant_ref(ins[i % P].data_ptr(), nbytes, a1.data_ptr(), nb, a2.data_ptr(), n2,
                                         outs[i % P].data_ptr(), _lib.BF16, m, n,
                                         torch.cuda.current_stream().cuda_stream) == 0
            t = graph_time(deq, 64)
            print(json.dumps({"m": m, "round": r, "variant": name, "us": round(t * 1e6, 3),
                              "TBps": round(nbytes * 5 / t / 1e12, 3)}), flush=True)
    del ins, outs
    torch.cuda.empty_cache()
