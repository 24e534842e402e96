"""Time grouped decode-GEMM launches (q/k/v and gate/up of Llama-3-8B) per cfg (diagnostic)."""
import argparse
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from nf4_triton_dequantization_amd import _lib  # noqa: E402
from sweep_gemm import graph_us  # noqa: E402

GROUPS = {"qkv": ([4096, 1024, 1024], 4096), "gateup": ([14336, 14336], 4096), "o": ([4096], 4096),
          "down": ([4096], 14336)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--cfg", action="append", default=[])
    ap.add_argument("--lib", default="prod")
    args = ap.parse_args()
    if args.lib != "prod":
        _lib.LIB_PATH = os.path.join(REPO, "tools", "_build", f"libnf4dq_{args.lib}.so")
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    M = args.m
    for name, (Ns, K) in GROUPS.items():
        wbytes = sum(n * K // 2 for n in Ns)
        copies = max(4, (640 << 20) // wbytes)
        sets = []
        for _ in range(copies):
            mats = (_lib.GemmMat * len(Ns))()
            keep = []
            for j, n in enumerate(Ns):
                nb = n * K // 64
                q = torch.randint(0, 256, (n * K // 2,), dtype=torch.uint8, device=dev)
                a1 = torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev)
                a2 = torch.rand((nb + 255) // 256, device=dev) * 0.01
                y = torch.empty((M, n), dtype=torch.bfloat16, device=dev)
                keep += [q, a1, a2, y]
                mats[j] = _lib.GemmMat(q.data_ptr(), q.numel(), a1.data_ptr(), nb, a2.data_ptr(), a2.numel(),
                                       y.data_ptr(), n)
            sets.append((mats, keep))
        x = torch.randn((M, K), device=dev).to(torch.bfloat16)
        for cs in ["default"] + args.cfg:
            cfg = None if cs == "default" else _lib.GemmCfg(*(int(v) for v in cs.split(",")))
            cp = ctypes.byref(cfg) if cfg is not None else None
            wsz = L.nf4_gemm_grouped_workspace_bytes(M, K, sets[0][0], len(Ns), cp)
            work = torch.zeros(max(wsz, 16), dtype=torch.uint8, device=dev)
            rc0 = L.nf4_gemm_ref_grouped(x.data_ptr(), M, K, sets[0][0], len(Ns), _lib.BF16, work.data_ptr(), wsz,
                                         cp, torch.cuda.current_stream().cuda_stream)
            if rc0 == _lib.ERR_ARG:
                continue

            def run(cp=cp, work=work, wsz=wsz):
                sp = torch.cuda.current_stream().cuda_stream
                for (mats, _k) in sets:
                    rc = L.nf4_gemm_ref_grouped(x.data_ptr(), M, K, mats, len(Ns), _lib.BF16, work.data_ptr(), wsz,
                                                cp, sp)
                    assert rc == 0, rc
            us = graph_us(run, copies)
            print(json.dumps({"group": name, "M": M, "cfg": cs, "us": round(us, 2),
                              "TBps": round(wbytes / us / 1e6, 3)}), flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
