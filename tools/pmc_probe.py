"""Workload for the PMC passes (run under rocprofv3 --pmc, see tools/pmc_traffic.py).

1. calibration: calib_read (1 GiB, 4 B/lane dword loads) and calib_write (1 GiB,
   16 B/lane nt stores) x 4 each -- known byte counts in the dequant kernel's
   two access shapes;
2. the bench workload: 4096x4096 NF4->bf16 dequant, bench.py's rotation (round 4:
   input and output sets rotated independently, >= 512 MiB of distinct reads and of
   writes, so the weights stream from HBM), 96 launches of the product entry; output
   dtype PMC_DTYPE (bf16, default, or f16).
"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from nf4_triton_dequantization_amd import _lib  # noqa: E402

CALIB_BYTES = 1 << 30


def main():
    m = int(os.environ.get("PMC_M", "4096"))
    n = int(os.environ.get("PMC_N", "4096"))
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    calib = ctypes.CDLL(os.path.join(REPO, "tools", "_build", "libpmccalib.so"))
    buf = torch.randint(0, 256, (CALIB_BYTES,), dtype=torch.uint8, device=dev)
    sink = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
    for _ in range(4):
        assert calib.calib_read(ctypes.c_void_p(buf.data_ptr()), ctypes.c_uint32(CALIB_BYTES),
                                ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(st)) == 0
    for _ in range(4):
        assert calib.calib_write(ctypes.c_void_p(buf.data_ptr()), ctypes.c_uint32(CALIB_BYTES),
                                 ctypes.c_void_p(st)) == 0
    torch.cuda.synchronize()
    del buf
    nb = m * n // 64
    n2 = (nb + 255) // 256
    sys.path.insert(0, REPO)
    import bench

    pin, pout = bench.rotation_sets([(0, m, n)])
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    ins = [(torch.randint(0, 256, (m * n // 2,), dtype=torch.uint8, device=dev, generator=g),
            torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=g),
            torch.rand(n2, device=dev, generator=g) * 0.01) for _ in range(pin)]
    f16 = os.environ.get("PMC_DTYPE", "bf16") == "f16"  # BASELINE configs[3]: the fp16 leg
    outs = [torch.empty((m, n), dtype=torch.float16 if f16 else torch.bfloat16, device=dev) for _ in range(pout)]
    L = _lib.lib()
    for i in range(96):
        q, a1, a2 = ins[i % pin]
        assert L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                 outs[i % pout].data_ptr(), _lib.F16 if f16 else _lib.BF16, m, n, st) == 0
    torch.cuda.synchronize()
    print("pmc probe done", m, n)


if __name__ == "__main__":
    main()
