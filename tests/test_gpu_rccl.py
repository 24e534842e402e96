"""The RCCL branch of the sharded path, on the one GPU a test box has (``-m gpu``).

SURVEY §8e / BASELINE configs[4]: quant statistics travel from the rank that loaded
them to the ranks that own the matrices; the data path has no collective.  The gloo
tests (test_dist_cpu.py) cover the multi-rank logic on CPU; this test runs the same
functions on the real backend: a world-size-1 ``nccl`` (= RCCL) process group bound to
``cuda:0`` (``init_process_group(device_id=...)``, as bench.py does), then
``scatter_quant_stats`` (``dist.scatter`` of device tensors), ``broadcast_quant_stats``
and ``max_over_ranks`` (``all_reduce`` MAX), and a dequant of the received statistics
against the C oracle.  It runs in a fresh child process, so the process group never
outlives the test and the parent's HIP state is untouched.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _child():
    import numpy as np
    import torch
    import torch.distributed as dist

    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import nf4_oracle as O
    from nf4_triton_dequantization_amd import _lib
    from nf4_triton_dequantization_amd.sharding import (QuantStats, broadcast_quant_stats, max_over_ranks,
                                                        scatter_quant_stats)

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res = {"backend": dist.get_backend()}
    try:
        shapes = [(64, 256), (128, 4096), (8, 11008)]
        host = []
        for i, (m, n) in enumerate(shapes):
            packed, a1, a2 = O.make_inputs(m, n, 77 + i, a2_kind="normal")
            host.append((packed, a1, a2, m, n))
        # rank 0 holds them on the device, as after loading a checkpoint
        src = [QuantStats(m, n, torch.from_numpy(a1).to(dev), torch.from_numpy(a2).to(dev),
                          [torch.bfloat16, torch.float16, torch.float32][i % 3])
               for i, (_, a1, a2, m, n) in enumerate(host)]
        got_s = scatter_quant_stats([src], dev, src=0)
        got_b = broadcast_quant_stats(src, dev, src=0)

        def same(got):
            return len(got) == len(src) and all(
                g.m == s.m and g.n == s.n and g.dtype == s.dtype and g.absmax.device == dev
                and g.absmax2.device == dev and torch.equal(g.absmax.cpu(), s.absmax.cpu())
                and torch.equal(g.absmax2.cpu().view(torch.int32), s.absmax2.cpu().view(torch.int32))
                for g, s in zip(got, src))

        res["scatter_equal"] = same(got_s)
        res["broadcast_equal"] = same(got_b)
        res["max"] = max_over_ranks(3.25, dev)
        # the received statistics drive the product kernel bit-exactly
        L = _lib.lib()
        ok = []
        for (packed, a1, a2, m, n), st in zip(host, got_s):
            q = torch.from_numpy(packed).to(dev)
            out = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
            rc = L.nf4_dequant_ref(q.data_ptr(), q.numel(), st.absmax.data_ptr(), st.absmax.numel(),
                                   st.absmax2.data_ptr(), st.absmax2.numel(), out.data_ptr(), _lib.BF16, m, n,
                                   torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            want = O.dequant_ref_np(packed, a1, a2, m, n, O.BF16)
            got = out.view(torch.int16).cpu().numpy().view(np.uint16)
            ok.append(rc == 0 and bool(np.array_equal(got, want)))
        res["dequant_equal"] = ok
    finally:
        dist.destroy_process_group()
    print("RESULT " + json.dumps(res), flush=True)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_rccl_world1_scatter_broadcast_max():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=220)
    assert p.returncode == 0, p.stderr[-4000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, p.stdout[-2000:] + p.stderr[-2000:]
    r = json.loads(line[-1][len("RESULT "):])
    assert r["backend"] == "nccl"
    assert r["scatter_equal"] and r["broadcast_equal"]
    assert r["max"] == 3.25
    assert r["dequant_equal"] == [True, True, True]


if __name__ == "__main__" and "--child" in sys.argv:
    _child()
