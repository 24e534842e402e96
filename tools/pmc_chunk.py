"""PMC workload for the chunk kernels' forms (tools only; run under rocprofv3 --pmc).

    PMC_CASE=chunk_4090 rocprofv3 --pmc FETCH_SIZE -d <dir> -o fetch --output-format csv -- python tools/pmc_chunk.py
    PMC_CASE=chunk_4090 rocprofv3 --pmc WRITE_SIZE -d <dir> -o write --output-format csv -- python tools/pmc_chunk.py
    PMC_KERNEL=nf4_chunk PMC_CASE=chunk_4090 python tools/pmc_traffic.py <dir> profiles/r06/chunk/pmc_chunk_4090.json

1. the calibration kernels of tools/pmc_probe.py (known byte counts in the flat kernel's
   access shapes: 4 B/lane dword loads, 16 B/lane nt stores), so pmc_traffic.py scales
   the counters the same way;
2. 64 launches of one case of tools/chunk_ab.py (PMC_CASE: chunk_4080 = the dense form,
   chunk_4090 / chunk_4095 = widths not a multiple of 8, pad_4096 = padded packed rows,
   unal_4096 = the packed weight at an odd address), bf16, HBM-streamed rotation.
"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from nf4_triton_dequantization_amd import _lib  # noqa: E402
from chunk_ab import SHAPES, case_sets  # noqa: E402

CALIB_BYTES = 1 << 30


def main():
    name = os.environ.get("PMC_CASE", "chunk_4090")
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
    m, n, flags = SHAPES[name]
    assert flags == 0, "the drop-in's own path only"
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    ins, outs = case_sets(name, dev, gen)
    L = _lib.lib()
    for i in range(64):
        q, a1, a2 = ins[i % len(ins)]
        o = outs[i % len(outs)]
        assert L.nf4_dequant_ref(q.data_ptr(), q.numel(), a1.data_ptr(), a1.numel(), a2.data_ptr(), a2.numel(),
                                 o.data_ptr(), _lib.BF16, m, n, st) == 0
    torch.cuda.synchronize()
    print("pmc chunk probe done", name, m, n)


if __name__ == "__main__":
    main()
