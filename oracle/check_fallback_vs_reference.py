"""Build-container check (needs /root/reference; never run on the GPU box):
oracle/fallback_torch.py vs the reference fallback ``_aggressive_pytorch_t4``
(kernel_optimized.py:208-314) on the C2 workload -- equal output bits, and
comparable CPU time (so bench.py's fallback figure stands for the reference's).

    PYTHONDONTWRITEBYTECODE=1 python oracle/check_fallback_vs_reference.py
"""
import os
import sys
import time
from types import SimpleNamespace

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")
sys.path.insert(0, HERE)
import fallback_torch as F  # noqa: E402
import nf4_oracle as O  # noqa: E402
from nf4_triton_dequantization.kernel_optimized import _aggressive_pytorch_t4  # noqa: E402


def main(m=4096, n=4096):
    p, a1, a2 = O.make_inputs(m, n, 3409)
    tp, ta1, ta2 = torch.from_numpy(p), torch.from_numpy(a1), torch.from_numpy(a2)
    qs = SimpleNamespace(absmax=ta1, state2=SimpleNamespace(absmax=ta2), dtype=torch.bfloat16)
    mod = SimpleNamespace(weight=SimpleNamespace(data=tp.view(-1, 1), quant_state=qs), out_features=m, in_features=n)
    runs = {"reference _aggressive_pytorch_t4": lambda: _aggressive_pytorch_t4(mod),
            "oracle/fallback_torch.py": lambda: F.dequant_fallback(tp, ta1, ta2, m, n, torch.bfloat16)}
    outs = {}
    for name, fn in runs.items():
        outs[name] = fn()
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        print(f"{name}: best of 3 {min(ts) * 1e3:.1f} ms ({torch.get_num_threads()} threads)")
    a, b = outs.values()
    print("outputs bit-equal:", torch.equal(a.view(torch.int16), b.view(torch.int16)))


if __name__ == "__main__":
    main()
