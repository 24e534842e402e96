"""Waves and threads past the end of a matrix (``-m gpu``).

Round 5's fuzzer (tools/fuzz_api.py seed 61) found a fault the suite had missed: in the
chunk kernel, a wave of the last workgroup lying wholly past the end of the matrix formed
its row index from its unclamped first chunk, gathered single-quant scales past the
absmax rows and wrote its (empty) staged span past the output.  This module sweeps that
class of shape on purpose, for every load / store form of the chunk kernels
(csrc/nf4_dequant.hip: the dense form; the general form -- rows < 512 -- with dword
loads or alignbyte dword pairs, whole-chunk 16-byte stores or LDS staging, rows of >= 64
chunks or fewer) and of the piece kernel (outputs in 16-byte pieces in output order: even
and odd n, padded rows, odd packed and output offsets, rows whose last block is shorter
than a piece; its fp32 form), in both scale modes:

* m is chosen so that the last workgroup (4 waves x 256 four-byte chunks, or 256 16-byte
  output pieces) holds 1, 2 and 3 waves wholly past the end, and 0 as the control;
* the absmax arrays have exactly the length the matrix needs -- nb = m * blocks per row,
  n2 = m * nested groups per row, single-quant rows of exactly blocks-per-row entries --
  so no modulo wrap keeps a runaway index inside them;
* 2^18-element sentinels after the output (and 64 before it) catch any write outside it.

The one-thread-per-byte kernels (nf4_rows_kernel, forced with NF4DQ_CFG_ROWS, and the
bitsandbytes nf4_bnb_bytes_kernel, which takes numel % 8 != 0) get the same treatment
with lengths that leave the last 256-thread workgroup partly empty.  Every output bit is
compared with the C oracle.
"""
import ctypes

import numpy as np
import pytest
import torch

import nf4_oracle as O
from _helpers import DT_CODE, check_guarded as _check, dev_bytes as _dev_bytes, out_buffer as _out_buffer

pytestmark = pytest.mark.gpu

# name: (n, extra packed bytes per row, packed byte offset, output element offset, dtypes, kernel)
FORMS = {
    "dense": (1000, 0, 0, 0, ("bf16", "f16"), "chunk"),              # n % 8 == 0, rows of exactly 4 L bytes
    "dword_whole": (504, 4, 0, 0, ("bf16", "f32"), "chunk"),         # padded rows: dword loads, 16-byte stores
    "alignbyte_whole": (504, 4, 1, 0, ("f16", "f32"), "chunk"),      # odd packed address, padded rows: dword pairs + v_alignbyte
    "dword_staged": (509, 1, 0, 0, ("bf16", "f16", "f32"), "chunk"),  # odd n, stride 256, L = 64: LDS-staged
    "alignbyte_staged": (510, 2, 0, 0, ("bf16", "f32"), "chunk"),    # stride 257, L = 64: both
    "unaligned_out": (504, 4, 0, 1, ("bf16",), "chunk"),             # padded rows, output one element off: staged
    "short_rows": (200, 0, 0, 0, ("bf16", "f32"), "chunk"),          # L = 25 < 64 chunks: per-step row division
    "short_odd": (77, 0, 0, 0, ("f16",), "chunk"),                   # L = 10, odd n: staged, dword pairs
    # the piece kernel (16-bit output, tight rows the dense form does not take):
    "piece_even": (1002, 0, 0, 0, ("bf16", "f16"), "piece"),         # the stream runs on across row ends
    "piece_odd": (1007, 0, 0, 0, ("bf16", "f16"), "piece"),          # a pad nibble at every row end
    "piece_offsets": (1007, 0, 1, 37, ("bf16",), "piece"),           # odd packed address, output 37 elements in
    "piece_aligned_n": (1000, 0, 0, 1, ("f16",), "piece"),           # n % 8 == 0, output one element off
    "piece_min_block": (520, 0, 3, 5, ("bf16",), "piece"),           # last block of 8 elements, rows of 520
    "piece_unal_packed": (1000, 0, 1, 0, ("f16",), "piece"),         # n % 8 == 0, aligned output, odd packed address
    "piece_tri": (1029, 0, 0, 0, ("bf16", "f16"), "piece"),          # last block of 5: three blocks in a piece
    "piece_padded": (1002, 4, 0, 0, ("bf16",), "piece"),             # padded rows: the next row's bytes apart
    "piece_padded_odd": (1007, 3, 1, 5, ("f16",), "piece"),
    # its fp32 form (4-element pieces; every tight fp32 shape the flat kernel does not take)
    "piece32_odd": (1007, 0, 1, 5, ("f32",), "piece32"),
    "piece32_even": (1002, 0, 0, 0, ("f32",), "piece32"),
    "piece32_aligned_n": (1000, 0, 0, 0, ("f32",), "piece32"),       # n % 8 == 0, everything aligned
    "piece32_tri": (1027, 0, 1, 3, ("f32",), "piece32"),             # last block of 3: three blocks in a piece
    "piece32_padded": (1002, 2, 0, 3, ("f32",), "piece32"),
}


def _chunks_per_row(n):
    return ((n + 1) // 2 + 3) // 4


def _units(form, m):
    """256 of these per wave: 4-byte packed chunks (chunk kernels) or 16-byte output pieces
    from the output's 128-byte line (the piece kernels; torch allocations are 128-aligned and
    the sentinel is 64 elements, so the output sits `ooff` elements into its line, modulo the
    line's 64 16-bit / 32 fp32 elements)."""
    n, _, _, ooff, _, kind = FORMS[form]
    if kind == "chunk":
        return m * _chunks_per_row(n)
    per = 8 if kind == "piece" else 4  # elements per 16-byte piece
    return -(-(ooff % (128 // (16 // per)) + m * n) // per)


def _m_with_past_end_waves(form, k, m0=1):
    """Smallest m >= m0 whose last workgroup holds exactly k waves wholly past the end."""
    for m in range(m0, 1 << 14):
        units = _units(form, m)
        waves = -(-units // 256)
        if 4 * -(-units // 1024) - waves == k:
            return m
    raise AssertionError((form, k))


def _exact_absmax(m, n, seed):
    bpr = (n + 63) // 64
    groups = (bpr + 3) // 4
    return {"nb": m * bpr, "n2": m * groups, "a2_kind": "normal"}, bpr


@pytest.mark.parametrize("form", sorted(FORMS))
@pytest.mark.parametrize("past", [0, 1, 2, 3])
@pytest.mark.parametrize("m0", [1, 300])  # one workgroup; many (the last one's rows deep in the matrix)
def test_chunk_forms_with_waves_past_the_end(coracle, gpu, form, past, m0):
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    n, pad, poff, ooff, dts, _ = FORMS[form]
    m = _m_with_past_end_waves(form, past, m0)
    seed = 7 * m + n + past
    ov, bpr = _exact_absmax(m, n, seed)
    stride = (n + 1) // 2 + pad
    p, a1, a2, single = O.golden_case_inputs(m, n, seed, dict(ov, stride=stride, single=0))
    assert a1.size == m * bpr and single.size == m * bpr
    st = torch.cuda.current_stream().cuda_stream
    pb, pp = _dev_bytes(p, gpu, poff)
    t1, t2, ts = (torch.from_numpy(a).to(gpu) for a in (a1, a2, single))
    for dt in dts:
        buf, start = _out_buffer(m, n, dt, gpu, ooff)
        assert buf.data_ptr() % 128 == 0  # (the piece count above assumes it)
        optr = buf.data_ptr() + start * buf.element_size()
        rc = L.nf4_dequant_ref(pp, p.size, t1.data_ptr(), t1.numel(), t2.data_ptr(), t2.numel(), optr, DT_CODE[dt],
                               m, n, st)
        assert rc == 0, rc
        torch.cuda.synchronize()
        _check(buf, start, m, n, dt, coracle.dequant_ref(p, a1, a2, m, n, DT_CODE[dt]),
               f"{form} ref {m}x{n} past {past} {dt}")
        buf, start = _out_buffer(m, n, dt, gpu, ooff)
        optr = buf.data_ptr() + start * buf.element_size()
        rc = L.nf4_dequant_single(pp, p.size, ts.data_ptr(), ts.numel(), optr, DT_CODE[dt], m, n, st)
        assert rc == 0, rc
        torch.cuda.synchronize()
        _check(buf, start, m, n, dt, coracle.dequant_single(p, single, m, n, DT_CODE[dt]),
               f"{form} single {m}x{n} past {past} {dt}")
    del pb


@pytest.mark.parametrize("m,n", [(1, 510), (3, 341), (5, 1000), (9, 77), (257, 3)])
def test_rows_kernel_partial_last_workgroup(coracle, gpu, m, n):
    """nf4_rows_kernel (NF4DQ_CFG_ROWS): one thread per packed byte; m * ceil(n/2) leaves the
    last 256-thread workgroup partly empty; exact-length absmax (the reference mode: the
    single-quant entry has no flag to force this kernel)."""
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    assert (m * ((n + 1) // 2)) % 256 != 0
    ov, _ = _exact_absmax(m, n, m + n)
    p, a1, a2, single = O.golden_case_inputs(m, n, m + n, dict(ov, stride=(n + 1) // 2, single=0))
    st = torch.cuda.current_stream().cuda_stream
    pb, pp = _dev_bytes(p, gpu)
    t1, t2 = torch.from_numpy(a1).to(gpu), torch.from_numpy(a2).to(gpu)
    cfg = _lib.LaunchCfg(4, 0, 1, _lib.CFG_ROWS)
    for dt in ("bf16", "f32"):
        buf, start = _out_buffer(m, n, dt, gpu, 0)
        rc = L.nf4_dequant_ref_cfg(pp, p.size, t1.data_ptr(), t1.numel(), t2.data_ptr(), t2.numel(),
                                   buf.data_ptr() + start * buf.element_size(), DT_CODE[dt], m, n, ctypes.byref(cfg), st)
        assert rc == 0, rc
        torch.cuda.synchronize()
        _check(buf, start, m, n, dt, coracle.dequant_ref(p, a1, a2, m, n, DT_CODE[dt]), f"rows {m}x{n} {dt}")
    del pb


@pytest.mark.parametrize("numel", [3, 1001, 4097, 64 * 257 + 5, 131073])
def test_bnb_bytes_kernel_partial_last_workgroup(coracle, gpu, numel):
    """nf4_bnb_bytes_kernel (bitsandbytes semantics, numel % 8 != 0): the last workgroup's
    threads past ceil(numel / 2) packed bytes idle; absmax arrays of exactly the block
    counts (nested and single-level), sentinels around the output."""
    from nf4_triton_dequantization_amd import _lib

    L = _lib.lib()
    assert numel % 8 != 0
    rng = np.random.default_rng(numel)
    nblk = -(-numel // 64)
    n2 = -(-nblk // 256)
    p = rng.integers(0, 256, (numel + 1) // 2, dtype=np.uint8)
    a1 = rng.integers(0, 256, nblk, dtype=np.uint8)
    code2 = np.sort(rng.uniform(-1, 1, 256).astype(np.float32))
    a2 = rng.uniform(1e-3, 1e-2, n2).astype(np.float32)
    single = rng.uniform(1e-3, 1.0, nblk).astype(np.float32)
    st = torch.cuda.current_stream().cuda_stream
    tp, t1, tc, t2, ts = (torch.from_numpy(a).to(gpu) for a in (p, a1, code2, a2, single))
    for dt in ("bf16", "f16", "f32"):
        buf, start = _out_buffer(1, numel, dt, gpu, 0)
        rc = L.nf4_dequant_bnb(tp.data_ptr(), t1.data_ptr(), nblk, tc.data_ptr(), t2.data_ptr(), n2, 0.03125,
                               buf.data_ptr() + start * buf.element_size(), DT_CODE[dt], numel, 64, 256, st)
        assert rc == 0, rc
        torch.cuda.synchronize()
        want = coracle.dequant_bnb(p, a1, code2, a2, 0.03125, numel, DT_CODE[dt])
        _check(buf, start, 1, numel, dt, np.asarray(want).reshape(1, numel), f"bnb {numel} {dt}")
        buf, start = _out_buffer(1, numel, dt, gpu, 0)
        rc = L.nf4_dequant_bnb_single(tp.data_ptr(), ts.data_ptr(), nblk, buf.data_ptr() + start * buf.element_size(),
                                      DT_CODE[dt], numel, 64, st)
        assert rc == 0, rc
        torch.cuda.synchronize()
        want = coracle.dequant_bnb_single(p, single, numel, DT_CODE[dt])
        _check(buf, start, 1, numel, dt, np.asarray(want).reshape(1, numel), f"bnb single {numel} {dt}")
