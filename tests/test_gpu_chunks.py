"""The chunk and piece kernels (``-m gpu``): every shape the flat kernel does not take.

n % 64 != 0, padded packed rows and unaligned pointers go through the kernels of
csrc/nf4_dequant.hip.  Which instantiation a shape takes (launch_chunks):
* nf4_chunk_dense_kernel -- 16-bit output, n % 8 == 0, packed rows of exactly 4 L bytes
  (L = chunks per row >= 64), 4-byte-aligned packed weight, 16-byte-aligned output;
* nf4_piece_kernel / nf4_piece32_kernel -- rows of n >= 512 that the dense form does not
  take (16-bit: n % 8 != 0, the output off 16-byte alignment or the packed weight off
  4-byte alignment, with tight or padded rows; fp32: every such shape): aligned 16-byte
  output pieces in output order, each from the two packed dwords around its nibbles
  (padded rows: a piece crossing its row's end loads the next row's first bytes apart);
* nf4_chunk_kernel<LW, SW> otherwise (rows < 512; 16-bit padded rows stored whole), with
  the load form LW = 4 (dword loads: packed weight and row stride 4-byte aligned) or 1
  (two aligned dwords per chunk joined with
  v_alignbyte: any alignment), and the store form SW = 16 (one 16-byte store per chunk,
  or two for fp32: n % 8 == 0 (fp32: n % 4 == 0) and a 16-byte-aligned output) or 4
  (16-bit outputs staged through LDS and written as aligned 16-byte pieces, the span's
  two end pieces element by element; fp32 stored one element at a time); rows of >= 64
  chunks advance their indices by additions, shorter ones divide per step.
These cases run every form through the C ABI in both scale modes and compare bit for bit
with the C oracle, with sentinels on both sides of the output (past-n pieces are dropped
by the buffer range, not branched around).  The NF4DQ_CFG_CHUNKS / NF4DQ_CFG_ROWS tuning
flags cross-check the chunk kernels against the flat kernel and the one-thread-per-byte
kernel.  Waves wholly past the end of a matrix: tests/test_gpu_edges.py.
"""
import ctypes

import numpy as np
import pytest
import torch

import nf4_oracle as O
from _helpers import DT_CODE, assert_bits_equal, check_guarded as _check, dev_bytes as _dev_bytes, out_bits
from _helpers import out_buffer as _out_buffer

pytestmark = pytest.mark.gpu


def _lib():
    from nf4_triton_dequantization_amd import _lib

    return _lib


def _ref_call(dev, p, a1, a2, m, n, dt, p_off=0, o_elem_off=0, flags=None):
    L = _lib().lib()
    pb, pp = _dev_bytes(p, dev, p_off)
    t1 = torch.from_numpy(a1).to(dev)
    t2 = torch.from_numpy(a2).to(dev)
    buf, start = _out_buffer(m, n, dt, dev, o_elem_off)
    optr = buf.data_ptr() + start * buf.element_size()
    st = torch.cuda.current_stream().cuda_stream
    if flags is None:
        rc = L.nf4_dequant_ref(pp, p.size, t1.data_ptr(), t1.numel(), t2.data_ptr(), t2.numel(), optr,
                               DT_CODE[dt], m, n, st)
    else:
        cfg = _lib().LaunchCfg(4, 0, 1, flags)
        rc = L.nf4_dequant_ref_cfg(pp, p.size, t1.data_ptr(), t1.numel(), t2.data_ptr(), t2.numel(), optr,
                                   DT_CODE[dt], m, n, ctypes.byref(cfg), st)
    assert rc == 0, rc
    torch.cuda.synchronize()
    del pb
    return buf, start


# (m, n, extra stride bytes, packed byte offset, output element offset): the form each
# selects for 16-bit output (fp32: the general form, SW 16 when n % 4 == 0 and aligned)
CASES = [
    (37, 1000, 0, 0, 0),      # n % 8 == 0, rows of exactly 4 L bytes, L >= 64: the dense form
    (5, 4080, 0, 0, 0),       # (the dense form)
    (33, 1000, 4, 0, 0),      # padded rows, n % 8 == 0: LW 4, SW 16 (fp32: the piece kernel)
    (33, 1002, 3, 0, 0),      # padded rows, n % 8 != 0: the piece kernel, next row's bytes loaded apart
    (33, 504, 4, 0, 0),       # padded rows < 512: LW 4 (dword loads), SW 16 (16-byte chunk stores), L < 64
    (33, 508, 4, 0, 0),       # LW 4, L >= 64: 16-bit SW 4 (staged), fp32 SW 16
    (9, 4080, 0, 0, 1),       # output off 16-byte alignment, tight rows: the piece kernel (fp32: LW 4, SW 4)
    (9, 4080, 4, 0, 1),       # the same with padded rows (piece kernel)
    (9, 510, 4, 0, 1),        # rows < 512, L >= 64, output off alignment: LW 4, SW 4 (staged)
    (9, 1002, 0, 0, 0),       # n % 8 == 2, stride 501: the piece kernel (fp32: LW 1, SW 4)
    (9, 1002, 1, 0, 0),       # n % 8 == 2, padded to stride 502 (piece kernel)
    (9, 506, 1, 0, 0),        # stride 254, L >= 64: LW 1, SW 4 (staged)
    (3, 6, 0, 0, 0),          # L = 1: LW 1, SW 4, per-step row division
    (7, 77, 0, 0, 0),         # odd n (stride 39): LW 1, SW 4
    (1, 1, 0, 0, 0),
    (4, 3, 0, 0, 0),
    (11, 200, 3, 0, 0),       # padded rows, stride % 4 != 0: LW 1, SW 16, L < 64
    (11, 200, 4, 0, 0),       # padded rows, stride % 4 == 0: LW 4, SW 16, L < 64
    (6, 256, 2, 0, 0),        # n % 64 == 0 but padded: not flat (LW 1)
    (6, 256, 0, 1, 0),        # odd packed pointer: LW 1
    (6, 256, 0, 2, 1),        # output one element off 16-byte alignment: SW 4
    (10, 1000, 0, 3, 3),      # piece kernel: odd packed address, output 3 elements off
    (10, 1000, 2, 3, 3),      # the same, padded rows (piece kernel)
    (10, 510, 2, 3, 3),       # rows < 512: LW 1, SW 4, L >= 64
    (3000, 2, 0, 0, 0),       # one chunk per row: 256 rows per wave (per-lane scale gathers)
    (300, 18, 5, 0, 1),
    (129, 4100, 4, 0, 0),     # padded rows, n % 64 == 4 (piece kernel, three blocks)
    (129, 509, 1, 0, 0),      # rows < 512, stride 256: LW 4, SW 4, partial last wave
    # the piece kernel: even n (the stream runs across row ends), odd n (a pad nibble per
    # row), the shortest last block it takes (8: n % 64 == 8), n % 64 == 0 with the output
    # off alignment, output offsets up to 63 elements into the first line, one row
    (9, 4090, 0, 0, 0),
    (9, 4095, 0, 0, 0),
    (7, 1007, 0, 1, 37),
    (5, 520, 0, 2, 63),
    (6, 4096, 0, 3, 5),
    (1, 600, 0, 0, 9),
    (70, 521, 0, 0, 0),       # rows of 521 (last block of 9): a step crosses a row end in most lanes
    (9, 4096, 0, 1, 0),       # n % 64 == 0, aligned output, odd packed address
    # rows whose last block is shorter than a piece (three blocks in one piece)
    (129, 4100, 0, 0, 0),
    (9, 4097, 0, 1, 3),
    (5, 577, 0, 2, 17),
    (8, 515, 0, 3, 1),
]


@pytest.mark.parametrize("dt", ["f16", "bf16", "f32"])
@pytest.mark.parametrize("m,n,pad,poff,ooff", CASES)
def test_chunk_kernel_forms_vs_oracle(coracle, gpu, dt, m, n, pad, poff, ooff):
    seed = 31 * m + n + pad + 7 * poff + 3 * ooff
    for ov in ({}, {"nb": 5, "n2": 3, "a2_kind": "normal"}):
        stride = (n + 1) // 2 + pad
        p, a1, a2, _ = O.golden_case_inputs(m, n, seed, dict(ov, stride=stride))
        want = coracle.dequant_ref(p, a1, a2, m, n, DT_CODE[dt])
        buf, start = _ref_call(gpu, p, a1, a2, m, n, dt, poff, ooff)
        _check(buf, start, m, n, dt, want, f"{m}x{n} pad {pad} poff {poff} ooff {ooff} {dt} {ov}")


@pytest.mark.parametrize("dt", ["f16", "bf16", "f32"])
def test_single_quant_chunk_kernel(coracle, gpu, dt):
    L = _lib().lib()
    # (48 x 269 and 51 x 275: the last workgroup has a wave wholly past the end, whose row
    # index once ran past the absmax rows -- an out-of-range gather, seen by fuzz_api seed 61;
    # 37 x 1000 and 5 x 4080 unpadded: the dense form's kSingle scale gather)
    for (m, n, extra, pad) in ((12, 200, 0, 0), (6, 1002, 3, 1), (33, 77, 1, 0), (5, 4080, 2, 4), (48, 269, 0, 0),
                               (51, 275, 2, 0), (122, 261, 1, 0), (37, 1000, 0, 0), (5, 4080, 1, 0),
                               (9, 4090, 0, 0), (7, 1007, 1, 0), (33, 521, 2, 0)):  # (the last three: piece kernel)
        stride = (n + 1) // 2 + pad
        p, _, _, single = O.golden_case_inputs(m, n, m + n, {"single": extra, "stride": stride})
        want = coracle.dequant_single(p, single, m, n, DT_CODE[dt])
        pb, pp = _dev_bytes(p, gpu)
        ts = torch.from_numpy(single).to(gpu)
        buf, start = _out_buffer(m, n, dt, gpu, 0)
        rc = L.nf4_dequant_single(pp, p.size, ts.data_ptr(), ts.numel(), buf.data_ptr() + start * buf.element_size(),
                                  DT_CODE[dt], m, n, torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()
        _check(buf, start, m, n, dt, want, f"single {m}x{n} pad {pad} {dt}")


@pytest.mark.parametrize("m,n", [(256, 1024), (1000, 4096), (7, 64)])
def test_chunk_kernel_equals_flat_kernel_on_flat_shapes(coracle, gpu, m, n):
    """NF4DQ_CFG_CHUNKS sends a flat-eligible matrix through the chunk kernel."""
    p, a1, a2, _ = O.golden_case_inputs(m, n, 900 + m, {"a2_kind": "normal"})
    want = coracle.dequant_ref(p, a1, a2, m, n, O.BF16)
    for flags in (0, _lib().CFG_CHUNKS, _lib().CFG_ROWS):
        buf, start = _ref_call(gpu, p, a1, a2, m, n, "bf16", flags=flags)
        _check(buf, start, m, n, "bf16", want, f"{m}x{n} flags {flags}")


@pytest.mark.parametrize("dt", ["f16", "f32"])
def test_rows_kernel_still_matches(coracle, gpu, dt):
    """NF4DQ_CFG_ROWS: the one-thread-per-byte kernel (past the chunk kernel's limits)."""
    for (m, n, pad) in ((9, 1002, 0), (7, 77, 0), (11, 200, 3)):
        p, a1, a2, _ = O.golden_case_inputs(m, n, m * n, {"stride": (n + 1) // 2 + pad, "nb": 11, "n2": 2})
        want = coracle.dequant_ref(p, a1, a2, m, n, DT_CODE[dt])
        buf, start = _ref_call(gpu, p, a1, a2, m, n, dt, flags=_lib().CFG_ROWS)
        _check(buf, start, m, n, dt, want, f"rows {m}x{n} {dt}")


@pytest.mark.parametrize("n,dt", [(4080, "bf16"), (4090, "bf16"), (4095, "f16"), (4100, "bf16"), (4090, "f32")])
def test_drop_in_takes_the_chunk_and_piece_kernels_for_odd_widths(coracle, gpu, n, dt):
    """The drop-in API on BASELINE-sized matrices with n % 64 != 0: 4080 the chunk kernel's
    dense form, the others the piece kernels (odd n: a pad nibble per row; 4100: a 4-element
    last block), bit for bit against the C oracle at full size."""
    import nf4_triton_dequantization as N
    from _helpers import make_module

    m = 4096
    p, a1, a2, _ = O.golden_case_inputs(m, n, n, {"stride": (n + 1) // 2})
    want = coracle.dequant_ref(p, a1, a2, m, n, DT_CODE[dt])
    out = N.triton_dequantize_nf4(make_module(p, a1, a2, m, n, dt, gpu))
    assert out.shape == (m, n) and out.is_contiguous()
    assert_bits_equal(out_bits(out), want, dt, f"drop-in {m}x{n} {dt}")
