"""Weight-stream load patterns of the fused GEMM, timed alone (tools/load_patterns.hip)."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from sweep_gemm import graph_us  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "_build", "libloadpat.so"))
lib.lp_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                          ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda", 0)
for (rows, k) in [(14336, 4096), (4096, 14336)]:
    rb = k // 2
    copies = max(8, (768 << 20) // (rows * rb))
    ws = [torch.randint(0, 256, (rows * rb,), dtype=torch.uint8, device=dev) for _ in range(copies)]
    out = torch.zeros(4, dtype=torch.int32, device=dev)
    for pat in (0, 3, 4):
        for depth in (2, 4):
            for parts in (2, 4, 8):
                def run(pat=pat, depth=depth, parts=parts):
                    sp = torch.cuda.current_stream().cuda_stream
                    for w in ws:
                        assert lib.lp_launch(pat, depth, w.data_ptr(), rows, rb, parts, out.data_ptr(), sp) == 0
                us = graph_us(run, copies)
                print(json.dumps({"rows": rows, "K": k, "pat": pat, "depth": depth, "parts": parts,
                                  "us": round(us, 2), "TBps": round(rows * rb / us / 1e6, 3)}), flush=True)
    del ws
