"""Correctness triage of the register-resident GEMM kernel over its configs (tools only).

For each (M, N, K) and each (waves, depth, chunk depth) the kernel's y is compared
with x @ W.t() in fp32, W written by the library's own nf4_dequant_ref; prints the
strips per workgroup the launch used and the worst relative error per config.
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nf4_triton_dequantization_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for (M, N, K) in [(16, 4160, 4096), (16, 2048, 4096), (1, 4160, 4096), (32, 4160, 4096), (16, 8192, 4096),
                      (16, 4160, 8192)]:
        q = torch.randint(0, 256, (N * K // 2,), dtype=torch.uint8, device=dev, generator=g)
        nb = N * K // 64
        a1 = torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
        a2 = torch.rand((nb + 255) // 256, device=dev, generator=g) * 0.01 + 1e-3
        W = torch.empty((N, K), dtype=torch.bfloat16, device=dev)
        assert L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), nb, a2.data_ptr(), a2.numel(), W.data_ptr(),
                                 _lib.BF16, N, K, torch.cuda.current_stream().cuda_stream) == 0
        x = torch.randn((M, K), device=dev, generator=g).to(torch.bfloat16)
        ref = x.float() @ W.float().t()
        for waves in (8, 16):
            for depth in (2, 4):
                for kpw in (1, 2, 4):
                    ks = -(-(K // 128) // (waves * kpw))
                    cfg = _lib.GemmCfg(_lib.GEMM_XR, waves, depth, ks, kpw)
                    wsz = L.nf4_gemm_workspace_bytes_cfg(M, N, K, ctypes.byref(cfg))
                    ws = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=dev)
                    y = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
                    rc = L.nf4_gemm_ref_cfg(x.data_ptr(), M, q.data_ptr(), q.numel(), a1.data_ptr(), nb, a2.data_ptr(),
                                            a2.numel(), y.data_ptr(), _lib.BF16, N, K, ws.data_ptr(), wsz,
                                            ctypes.byref(cfg), torch.cuda.current_stream().cuda_stream)
                    torch.cuda.synchronize()
                    if rc:
                        print(json.dumps({"M": M, "N": N, "K": K, "cfg": [waves, depth, ks, kpw], "rc": rc}))
                        torch.cuda.synchronize()
                        continue
                    err = ((y.float() - ref).abs() / (ref.abs() + 1.0)).nan_to_num(1e9)
                    bad = (err > 0.02).nonzero()
                    wg_per_cu = 1 if waves == 16 or kpw == 2 else 2
                    P = max(1, cus * wg_per_cu // ks)
                    per_strip = (err > 0.02).reshape(M, N // 16, 16).any(dim=2).any(dim=0).nonzero().flatten()
                    print(json.dumps({"M": M, "N": N, "K": K, "cfg": [waves, depth, ks, kpw],
                                      "bad_strips_head": per_strip[:24].tolist(), "n_bad_strips": int(per_strip.numel()),
                                      "strips_per_wg_est": -(-(N // 16) // P), "max_err": float(err.max()),
                                      "bad": int(bad.shape[0]),
                                      "first_bad_col": int(bad[:, 1].min()) if bad.shape[0] else None}), flush=True)


if __name__ == "__main__":
    main()
