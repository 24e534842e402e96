"""Prequantized NF4 safetensors (bitsandbytes / transformers key layout): write, read, dequantize."""
import json

import numpy as np
import pytest
import torch

import nf4_oracle as O
from nf4_triton_dequantization_amd.bnb_layout import quantize_nf4
from nf4_triton_dequantization_amd.checkpoint import (QS_SUFFIX, load_nf4_safetensors, quant_state_tensors,
                                                      save_nf4_safetensors)

# the key patterns transformers' Bnb4bitDeserialize consumes (quantizer_bnb_4bit.py)
TRANSFORMERS_PATTERNS = {"weight.nested_absmax", "weight.nested_quant_map", "weight.quant_map", "weight.absmax",
                         "weight.quant_state.bitsandbytes__nf4", "weight"}


def _weights():
    torch.manual_seed(3)
    out = {}
    for name, (m, n, nested, dt) in {"model.layers.0.mlp.up_proj": (256, 512, True, torch.bfloat16),
                                     "model.layers.0.self_attn.k_proj": (64, 512, True, torch.float16),
                                     "lm_head": (96, 256, False, torch.bfloat16)}.items():
        w = torch.randn(m, n) * 0.02
        packed, qs = quantize_nf4(w, compress_statistics=nested)
        qs.dtype = dt
        out[name + ".weight"] = (packed, qs)
    return out


def test_keys_follow_transformers_layout():
    (packed, qs), = [_weights()["model.layers.0.mlp.up_proj.weight"]]
    t = quant_state_tensors("x.weight", packed, qs)
    assert {k[len("x."):] for k in t} == TRANSFORMERS_PATTERNS
    meta = json.loads(bytes(t["x.weight." + QS_SUFFIX].tolist()).decode())
    assert meta["quant_type"] == "nf4" and meta["blocksize"] == 64 and meta["nested_blocksize"] == 256
    assert meta["dtype"] == "bfloat16" and meta["shape"] == [256, 512] and meta["nested_dtype"] == "float32"
    assert t["x.weight"].dtype == torch.uint8 and t["x.weight.absmax"].dtype == torch.uint8


def test_roundtrip(tmp_path):
    ws = _weights()
    path = str(tmp_path / "nf4.safetensors")
    save_nf4_safetensors(path, ws)
    mods = load_nf4_safetensors(path)
    assert set(mods) == {k[: -len(".weight")] for k in ws}
    for prefix, (packed, qs) in ws.items():
        mod = mods[prefix[: -len(".weight")]]
        q2 = mod.weight.quant_state
        assert torch.equal(mod.weight.data, packed)
        assert mod.out_features == qs.shape[0] and mod.in_features == qs.shape[1]
        assert torch.equal(q2.absmax, qs.absmax) and q2.dtype == qs.dtype and q2.blocksize == qs.blocksize
        assert torch.equal(q2.code, qs.code)
        if qs.state2 is not None:
            assert torch.equal(q2.state2.absmax, qs.state2.absmax)
            assert torch.equal(q2.state2.code, qs.state2.code)
            assert float(q2.offset) == pytest.approx(float(qs.offset), rel=0, abs=0)
        else:
            assert q2.state2 is None


def test_mixed_checkpoint_reads_only_nf4_entries(tmp_path, monkeypatch):
    """A checkpoint also holding unquantized tensors (embeddings, norms): only the NF4
    weights become modules, and only their entries are read from the file."""
    from safetensors import safe_open
    from safetensors.torch import save_file

    from nf4_triton_dequantization_amd.checkpoint import quant_state_tensors

    ws = _weights()
    tensors = {}
    for prefix, (packed, qs) in ws.items():
        tensors.update(quant_state_tensors(prefix, packed, qs))
    tensors["model.embed_tokens.weight"] = torch.randn(64, 32)
    tensors["model.norm.weight"] = torch.ones(32)
    path = str(tmp_path / "mixed.safetensors")
    save_file(tensors, path)
    read = []
    real_open = safe_open

    class _Spy:
        def __init__(self, *a, **k):
            self._f = real_open(*a, **k)

        def __enter__(self):
            self._f.__enter__()
            return self

        def __exit__(self, *exc):
            return self._f.__exit__(*exc)

        def keys(self):
            return self._f.keys()

        def get_tensor(self, k):
            read.append(k)
            return self._f.get_tensor(k)

    import safetensors

    monkeypatch.setattr(safetensors, "safe_open", _Spy)
    mods = load_nf4_safetensors(path)
    assert set(mods) == {k[: -len(".weight")] for k in ws}
    assert "model.embed_tokens.weight" not in read and "model.norm.weight" not in read
    assert set(read) == set(tensors) - {"model.embed_tokens.weight", "model.norm.weight"}


@pytest.mark.gpu
def test_loaded_checkpoint_dequantizes_on_gpu(tmp_path, coracle, gpu):
    from nf4_triton_dequantization import triton_dequantize_nf4
    from nf4_triton_dequantization_amd import dequantize_nf4_bnb

    ws = _weights()
    path = str(tmp_path / "nf4.safetensors")
    save_nf4_safetensors(path, ws)
    for name, mod in load_nf4_safetensors(path, device=gpu).items():
        packed, qs = ws[name + ".weight"]
        m, n = qs.shape
        p = packed.view(-1).numpy()
        dt = O.BF16 if qs.dtype == torch.bfloat16 else O.F16
        got = dequantize_nf4_bnb(mod).contiguous().view(torch.int16).cpu().numpy().view(np.uint16)
        if qs.state2 is not None:
            want = coracle.dequant_bnb(p, qs.absmax.numpy(), qs.state2.code.numpy(), qs.state2.absmax.numpy(),
                                       float(qs.offset), m * n, dt).reshape(m, n)
            # reference semantics straight from the same module (the drop-in entry point)
            ref = triton_dequantize_nf4(mod).contiguous().view(torch.int16).cpu().numpy().view(np.uint16)
            assert np.array_equal(ref, coracle.dequant_ref(p, qs.absmax.numpy(), qs.state2.absmax.numpy(), m, n, dt))
        else:
            want = coracle.dequant_bnb_single(p, qs.absmax.numpy(), m * n, dt).reshape(m, n)
        assert np.array_equal(got, want), name
