"""Proof that a split-K timeout is reported, not silent.

    NF4DQ_LIB_PATH=tools/_build/libnf4dq_abl_dropslice.so python tools/splitk_timeout_probe.py

Runs ONE 128-deep-kernel GEMM with 4 K slices on the drop-slice ablation build
(tools/gemm_ablate.hip ABL_DROPSLICE: slice 1 takes its ticket but never stores
its partials), so the reducer's bounded poll gives up.  Expected, and printed as
one JSON line: the launch returns OK, the missing slice's outputs are NaN,
nf4_gemm_check_workspace returns NF4DQ_ERR_SPLITK_TIMEOUT and leaves the
workspace zero-filled, and a second check returns OK.  Then the same call on the
product library (no NF4DQ_LIB_PATH) returns a finite y and a clean check.  One run
by design -- never loop it.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import workloads as W  # noqa: E402
from nf4_triton_dequantization_amd import _lib  # noqa: E402


def main():
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    M, N, K = 4, 256, 1024
    p, a1, a2 = W.make_inputs(N, K, 11)
    gp, ga1, ga2 = (torch.from_numpy(v).to(dev) for v in (p, a1, a2))
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    y = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
    cfg = _lib.GemmCfg(_lib.GEMM_K128, 4, 1, 4, 1)  # 4 K slices over workgroups: ticket + poll hand-off
    wsz = L.nf4_gemm_workspace_bytes_cfg(M, N, K, ctypes.byref(cfg))
    ws = torch.zeros(wsz, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    rc = L.nf4_gemm_ref_cfg(x.data_ptr(), M, gp.data_ptr(), p.size, ga1.data_ptr(), a1.size, ga2.data_ptr(), a2.size,
                            y.data_ptr(), _lib.BF16, N, K, ws.data_ptr(), wsz, ctypes.byref(cfg), st)
    chk = L.nf4_gemm_check_workspace(ws.data_ptr(), wsz, st)
    torch.cuda.synchronize()
    res = {"lib": os.path.basename(_lib.LIB_PATH), "M": M, "N": N, "K": K, "ksplit": 4, "launch_rc": rc,
           "check_rc": chk, "check_msg": _lib.strerror(chk), "nan_outputs": int(torch.isnan(y.float()).sum()),
           "workspace_nonzero_after_check": int(ws.count_nonzero()),
           "second_check_rc": L.nf4_gemm_check_workspace(ws.data_ptr(), wsz, st)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
