"""Does buffer placement move the 4096^2 dequant time?  (diagnostic)

Allocates bench.py's 16 buffer sets after a dummy allocation of varying size,
times the same hipGraph replay each time, and prints us/step per placement.
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from nf4_triton_dequantization_amd import _lib  # noqa: E402

L = _lib.lib()
dev = torch.device("cuda", 0)
m = n = 4096
nb, n2 = m * n // 64, m * n // 64 // 256
for pad_mb in [0, 1, 2, 3, 5, 8, 13, 0, 1, 2]:
    pad = torch.empty(pad_mb << 20, dtype=torch.uint8, device=dev) if pad_mb else None
    sets = [(torch.randint(0, 256, (m * n // 2,), dtype=torch.uint8, device=dev),
             torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev),
             torch.rand(n2, device=dev) * 0.01 + 1e-3,
             torch.empty((m, n), dtype=torch.bfloat16, device=dev)) for _ in range(16)]
    st = torch.cuda.current_stream()

    def step(i):
        q, a1, a2, o = sets[i % 16]
        sp = torch.cuda.current_stream().cuda_stream  # the capture stream inside torch.cuda.graph
        assert L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), nb, a2.data_ptr(), n2, o.data_ptr(),
                                 _lib.BF16, m, n, sp) == 0
    for i in range(20):
        step(i)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(200):
            step(i)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / 200)
    ts.sort()
    addr = [(s[0].data_ptr() >> 20, s[3].data_ptr() >> 20) for s in sets[:3]]
    print(json.dumps({"pad_mb": pad_mb, "us": [round(t, 3) for t in ts], "first_sets_MiB": addr}), flush=True)
    del sets, g, pad
    torch.cuda.empty_cache()
