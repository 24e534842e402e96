"""C-ABI library: loads, exports every symbol include/nf4_dequant.h declares, and
rejects bad arguments on the host before any device work (no GPU needed)."""
import ctypes
import re

import pytest

from nf4_triton_dequantization_amd import _lib


def _header_functions():
    text = open(_lib.HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(nf4_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_expected_entry_points():
    fns = _header_functions()
    for name in ("nf4_dequant_ref", "nf4_dequant_single", "nf4_dequant_ref_batched", "nf4_dequant_bnb",
                 "nf4_dequant_bnb_single", "nf4_dequant_ref_cfg", "nf4_strerror", "nf4_version"):
        assert name in fns


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in _header_functions():
        assert hasattr(L, name), name
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"


_CTYPE_OF = {  # C parameter / return type in the header -> the ctypes type the binding must use
    "int": ctypes.c_int, "int32_t": ctypes.c_int32, "int64_t": ctypes.c_int64, "size_t": ctypes.c_size_t,
    "float": ctypes.c_float, "void*": ctypes.c_void_p, "const void*": ctypes.c_void_p,
    "const uint8_t*": ctypes.c_void_p, "const float*": ctypes.c_void_p, "const char*": ctypes.c_char_p,
    "const nf4_matrix_desc*": ctypes.POINTER(_lib.MatrixDesc), "const nf4_launch_cfg*": ctypes.POINTER(_lib.LaunchCfg),
    "const nf4_gemm_cfg*": ctypes.POINTER(_lib.GemmCfg), "const nf4_gemm_mat*": ctypes.POINTER(_lib.GemmMat),
}


def _header_prototypes():
    """name -> (return C type, [parameter C types]) for every prototype of the header."""
    text = re.sub(r"/\*.*?\*/", "", open(_lib.HEADER_PATH).read(), flags=re.S)
    protos = {}
    for ret, name, params in re.findall(r"^\s*((?:const\s+)?\w+\s*\*?)\s*(nf4_\w+)\s*\(([^)]*)\)\s*;", text,
                                        flags=re.M):
        types = []
        for p in [p.strip() for p in params.split(",") if p.strip() and p.strip() != "void"]:
            p = re.sub(r"\s*\*\s*", "* ", p)           # "T *x" / "T* x" -> "T* x"
            types.append(p.rsplit(" ", 1)[0].strip())  # drop the parameter name
        protos[name] = (re.sub(r"\s*\*", "*", ret.strip()), types)
    return protos


def test_binding_argtypes_equal_header_prototypes():
    """Every exported entry's ctypes restype/argtypes are exactly the header's C types,
    parameter by parameter (a drifted binding would pass wrong-width integers)."""
    protos = _header_prototypes()
    assert sorted(protos) == _header_functions()
    for name, (ret, params) in protos.items():
        res, args = _lib.SIGNATURES[name]
        assert res == _CTYPE_OF[ret], (name, ret, res)
        assert len(args) == len(params), (name, params, args)
        for i, (c, t) in enumerate(zip(params, args)):
            assert t == _CTYPE_OF[c], (name, i, c, t)
        fn = getattr(_lib.lib(), name)
        assert fn.restype == res and list(fn.argtypes) == list(args), name


def test_survey_8b_signature_departure_is_packed_len_only():
    """SURVEY §8(b) specifies nf4_dequant_ref(packed, absmax_q, nb, absmax2, n2, out,
    out_dtype, m, n, hip_stream).  The header adds exactly one parameter, `packed_len`
    after `packed` (the reference's `.view(m, -1)` row stride, kernel_optimized.py:229),
    and the departure is recorded in the header itself."""
    survey = ["const uint8_t*", "const uint8_t*", "int64_t", "const float*", "int64_t", "void*", "int32_t",
              "int64_t", "int64_t", "void*"]
    _, params = _header_prototypes()["nf4_dequant_ref"]
    assert params[:1] + params[2:] == survey and params[1] == "int64_t"
    _, cpu = _header_prototypes()["nf4_dequant_ref_cpu"]
    assert cpu[:-1] == params[:-1] and cpu[-1] == "int32_t"  # host form: `threads` for the stream
    text = open(_lib.HEADER_PATH).read()
    assert "Departure from SURVEY.md §8(b)" in text and "packed_len" in text


def test_header_constants_match_binding():
    text = open(_lib.HEADER_PATH).read()
    consts = dict(re.findall(r"#define\s+(NF4DQ_\w+)\s+(\d+)", text))
    assert int(consts["NF4DQ_F16"]) == _lib.F16
    assert int(consts["NF4DQ_BF16"]) == _lib.BF16
    assert int(consts["NF4DQ_F32"]) == _lib.F32
    assert int(consts["NF4DQ_ERR_ARG"]) == _lib.ERR_ARG
    assert int(consts["NF4DQ_ERR_SHAPE"]) == _lib.ERR_SHAPE
    assert int(consts["NF4DQ_BATCH_MAX"]) == _lib.BATCH_MAX
    assert int(consts["NF4DQ_ERR_SPLITK_TIMEOUT"]) == _lib.ERR_SPLITK_TIMEOUT


def test_struct_layouts():
    assert ctypes.sizeof(_lib.MatrixDesc) == 9 * 8
    assert ctypes.sizeof(_lib.LaunchCfg) == 16


def test_version_and_strerror():
    L = _lib.lib()
    assert b"gfx950" in L.nf4_version()
    assert L.nf4_strerror(0) == b"ok"
    assert b"shape" in L.nf4_strerror(2)
    assert b"split-K" in L.nf4_strerror(_lib.ERR_SPLITK_TIMEOUT)


def test_check_workspace_host_validation():
    """nf4_gemm_check_workspace: nothing to report without a workspace; a buffer too
    small to hold the header was never a split-K workspace (host checks, no device call)."""
    L = _lib.lib()
    assert L.nf4_gemm_check_workspace(None, 0, None) == _lib.OK
    assert L.nf4_gemm_check_workspace(FAKE, 1024, None) == _lib.ERR_ARG


def test_check_gemm_workspaces_without_workspaces():
    """The Python check has nothing to report before any fused-GEMM call (no device call)."""
    from nf4_triton_dequantization_amd import check_gemm_workspaces, kernel

    saved = dict(kernel._GEMM_WS)
    kernel._GEMM_WS.clear()
    try:
        assert check_gemm_workspaces() is None
    finally:
        kernel._GEMM_WS.update(saved)


FAKE = 0x1000  # never dereferenced: every call below fails validation first


@pytest.mark.parametrize("args,want", [
    # bad dtype
    ((FAKE, 64, FAKE, 2, FAKE, 1, FAKE, 7, 2, 64, None), _lib.ERR_ARG),
    # negative m
    ((FAKE, 64, FAKE, 2, FAKE, 1, FAKE, 0, -1, 64, None), _lib.ERR_ARG),
    # packed_len not divisible by m (view(m, -1) fails, kernel_optimized.py:229)
    ((FAKE, 65, FAKE, 2, FAKE, 1, FAKE, 1, 2, 64, None), _lib.ERR_SHAPE),
    # packed rows shorter than ceil(n/2)
    ((FAKE, 60, FAKE, 2, FAKE, 1, FAKE, 1, 2, 64, None), _lib.ERR_SHAPE),
    # empty absmax
    ((FAKE, 64, FAKE, 0, FAKE, 1, FAKE, 1, 2, 64, None), _lib.ERR_ARG),
    # null output
    ((FAKE, 64, FAKE, 2, FAKE, 1, None, 1, 2, 64, None), _lib.ERR_ARG),
    # empty matrix: nothing to do, nothing launched
    ((None, 0, None, 0, None, 0, None, 1, 0, 64, None), _lib.OK),
    ((None, 0, None, 0, None, 0, None, 1, 5, 0, None), _lib.OK),
])
def test_ref_validation(args, want):
    assert _lib.lib().nf4_dequant_ref(*args) == want


def test_single_validation():
    L = _lib.lib()
    # absmax cannot be viewed as (m, -1)
    assert L.nf4_dequant_single(FAKE, 64, FAKE, 3, FAKE, 1, 2, 64, None) == _lib.ERR_SHAPE
    # absmax rows shorter than blocks per row
    assert L.nf4_dequant_single(FAKE, 128, FAKE, 2, FAKE, 1, 2, 128, None) == _lib.ERR_SHAPE


def test_bnb_validation():
    L = _lib.lib()
    # blocksize not a power of two / below 64
    assert L.nf4_dequant_bnb(FAKE, FAKE, 4, FAKE, FAKE, 1, 0.0, FAKE, 1, 256, 96, 256, None) == _lib.ERR_ARG
    assert L.nf4_dequant_bnb(FAKE, FAKE, 8, FAKE, FAKE, 1, 0.0, FAKE, 1, 256, 32, 256, None) == _lib.ERR_ARG
    # too few absmax blocks
    assert L.nf4_dequant_bnb(FAKE, FAKE, 3, FAKE, FAKE, 1, 0.0, FAKE, 1, 256, 64, 256, None) == _lib.ERR_SHAPE
    # too few nested absmax
    assert L.nf4_dequant_bnb(FAKE, FAKE, 600, FAKE, FAKE, 2, 0.0, FAKE, 1, 600 * 64, 64, 256, None) == _lib.ERR_SHAPE
    assert L.nf4_dequant_bnb_single(FAKE, FAKE, 3, FAKE, 1, 256, 64, None) == _lib.ERR_SHAPE
    assert L.nf4_dequant_bnb_single(None, None, 0, None, 1, 0, 64, None) == _lib.OK


def test_batched_validation():
    L = _lib.lib()
    d = (_lib.MatrixDesc * 2)(_lib.MatrixDesc(FAKE, 64, FAKE, 2, FAKE, 1, FAKE, 2, 64),
                              _lib.MatrixDesc(FAKE, 65, FAKE, 2, FAKE, 1, FAKE, 2, 64))
    # the second descriptor is invalid: nothing is launched, the error is reported
    assert L.nf4_dequant_ref_batched(d, 2, 1, None) == _lib.ERR_SHAPE
    assert L.nf4_dequant_ref_batched(d, 1, 9, None) == _lib.ERR_ARG
    assert L.nf4_dequant_ref_batched(None, 0, 1, None) == _lib.OK


def test_cfg_validation():
    L = _lib.lib()
    cfg = _lib.LaunchCfg(3, 0, 0, 0)
    assert L.nf4_dequant_ref_cfg(FAKE, 64, FAKE, 2, FAKE, 1, FAKE, 1, 2, 64, ctypes.byref(cfg), None) == _lib.ERR_ARG
    # only tile_dwords 4, nontemporal 1 and a grid cap >= 0 remain; flags is 0, NF4DQ_CFG_ROWS or
    # NF4DQ_CFG_CHUNKS (not both, no other bit)
    assert (_lib.CFG_ROWS, _lib.CFG_CHUNKS) == (1, 2)
    for bad in ((8, 0, 1, 0), (2, 0, 1, 0), (4, 0, 0, 0), (4, -1, 1, 0), (4, 0, 1, 3), (4, 0, 1, 4), (4, 0, 1, 0x8),
                (4, 0, 1, 0x100), (4, 0, 1, 0x2000), (4, 0, 1, 0x10000)):
        cfg = _lib.LaunchCfg(*bad)
        assert L.nf4_dequant_ref_cfg(FAKE, 64, FAKE, 2, FAKE, 1, FAKE, 1, 2, 64, ctypes.byref(cfg), None) == \
            _lib.ERR_ARG, bad


def test_tensor_fast_entry_loads_and_declines_host_tensors():
    """csrc/nf4_torch_ext.cpp is built in-tree and loads beside libnf4dq.so; host
    tensors (and anything else off its fast path) come back as None, never computed."""
    import torch

    from nf4_triton_dequantization_amd import kernel

    E = _lib.ext()
    assert E is not None and kernel._ext() is E
    q = torch.zeros(64, dtype=torch.uint8)
    assert E.dequant_ref(q, torch.ones(2, dtype=torch.uint8), torch.ones(1), 2, 64, _lib.BF16) is None


def _run_py(code, **env):
    import os
    import subprocess
    import sys

    e = dict(os.environ, **env)
    return subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=120,
                          cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_import_without_library_then_loud_failure():
    """Importing the package loads no native code: the pure-Python helpers (quantizer,
    checkpoint layout) work without libnf4dq.so, and the first compute call raises."""
    code = (
        "import torch, types\n"
        "import nf4_triton_dequantization_amd as P\n"
        "from nf4_triton_dequantization_amd import bnb_layout\n"
        "w = torch.randn(4, 64)\n"
        "bnb_layout.quantize_nf4(w)\n"
        "from nf4_triton_dequantization import triton_dequantize_nf4\n"
        "qs = types.SimpleNamespace(absmax=torch.zeros(4, dtype=torch.uint8), dtype=torch.bfloat16,\n"
        "    state2=types.SimpleNamespace(absmax=torch.ones(1)))\n"
        "mod = types.SimpleNamespace(weight=types.SimpleNamespace(data=torch.zeros(128, 1, dtype=torch.uint8),\n"
        "    quant_state=qs), out_features=4, in_features=64)\n"
        "try:\n"
        "    triton_dequantize_nf4(mod)\n"
        "except RuntimeError as e:\n"
        "    assert 'not built' in str(e), e\n"
        "    print('raised')\n"
    )
    r = _run_py(code, NF4DQ_LIB_PATH="/nonexistent/libnf4dq.so")
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "raised"


def test_diagnostic_lib_path_skips_tensor_entry():
    """With NF4DQ_LIB_PATH set, nf4ext.so (linked to the product build) is not loaded,
    so every call goes to the selected build; a broken ext file only warns."""
    r = _run_py("from nf4_triton_dequantization_amd import _lib; print(_lib.ext())",
                NF4DQ_LIB_PATH=_lib.LIB_PATH)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "None"
