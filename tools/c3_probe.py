"""Where does the batched Llama pass (c3) lose against one big matrix?  Diagnostic.

    python tools/c3_probe.py

Times (HIP events, median of 5) the 224-weight Llama-3-8B pass three ways:
batched C ABI (<= NF4DQ_BATCH_MAX per launch), one launch per weight captured
in a hipGraph, and a single matrix of the same total size class (32768 x 16384,
one launch) as the steady-state reference.
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from bench_configs import LLAMA3_8B, alg_bytes, make_weight, timed  # noqa: E402
from nf4_triton_dequantization_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    ws = [make_weight(m, n, dev, gen, torch.bfloat16) for _ in range(32) for (m, n) in LLAMA3_8B]
    byt = sum(alg_bytes(o.shape[0], o.shape[1], 2) for *_, o in ws)
    descs = (_lib.MatrixDesc * len(ws))(*[
        _lib.MatrixDesc(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                        o.data_ptr(), o.shape[0], o.shape[1]) for (q, a1, a2, o) in ws])

    def batched():
        assert L.nf4_dequant_ref_batched(descs, len(ws), _lib.BF16, torch.cuda.current_stream().cuda_stream) == 0

    def singles():
        sp = torch.cuda.current_stream().cuda_stream
        for (q, a1, a2, o) in ws:
            assert L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                     o.data_ptr(), _lib.BF16, o.shape[0], o.shape[1], sp) == 0

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        singles()
    gb = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gb):
        batched()
    for name, fn in (("batched eager", batched), ("batched graph", gb.replay), ("224 single launches, graph", g.replay)):
        t = timed(fn, 5)
        print(json.dumps({"c3": name, "ms": t * 1e3, "GBps": byt / t / 1e9, "frac": byt / t / 8e12}), flush=True)
    del ws, descs
    torch.cuda.empty_cache()
    for (m, n) in ((32768, 16384), (16384, 16384), (8192, 8192)):
        sets = max(2, (1 << 30) // (m * n // 2 * 5))
        big = [make_weight(m, n, dev, gen, torch.bfloat16) for _ in range(sets)]
        i = [0]

        def one():
            q, a1, a2, o = big[i[0] % sets]
            i[0] += 1
            assert L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                     o.data_ptr(), _lib.BF16, m, n, torch.cuda.current_stream().cuda_stream) == 0
        t = timed(one, 7)
        b = alg_bytes(m, n, 2)
        print(json.dumps({"single": f"{m}x{n}", "sets": sets, "us": t * 1e6, "GBps": b / t / 1e9, "frac": b / t / 8e12}),
              flush=True)
        del big
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
