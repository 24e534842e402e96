"""Prequantized NF4 checkpoints in the bitsandbytes / transformers safetensors layout.

SURVEY §8f row 3.  A bnb-quantized ``Linear4bit`` named ``<prefix>`` is stored as
(the key set transformers' ``Bnb4bitDeserialize`` consumes; in-container source:
transformers/quantizers/quantizer_bnb_4bit.py ``get_weight_conversions``)::

    <prefix>.weight                                   uint8 [numel/2, 1] packed codes
    <prefix>.weight.absmax                            uint8 (nested) or fp32 absmax
    <prefix>.weight.quant_map                         fp32 [16] NF4 code book
    <prefix>.weight.nested_absmax                     fp32 state2.absmax      (nested only)
    <prefix>.weight.nested_quant_map                  fp32 [256] state2.code  (nested only)
    <prefix>.weight.quant_state.bitsandbytes__nf4     uint8 = UTF-8 JSON of the non-tensor fields:
        {"quant_type", "blocksize", "dtype", "shape", "nested_blocksize", "nested_dtype", "nested_offset"}

(bitsandbytes' ``QuantState.as_dict(packed=True)`` writes exactly this; the
library itself is absent here, so byte-for-byte compatibility with files it
wrote is unpinned -- the tests pin our writer/reader round trip and the key set.)

Loading uses ``safetensors`` only (no pickle) and yields ``Linear4bit``-layout
modules that ``triton_dequantize_nf4`` / ``dequantize_nf4_bnb`` accept directly.
"""
from __future__ import annotations

import json
from typing import Dict, Tuple

import torch

from .bnb_layout import Linear4bit, Params4bit, QuantState

QS_SUFFIX = "quant_state.bitsandbytes__nf4"
_DT_NAMES = {"float16": torch.float16, "bfloat16": torch.bfloat16, "float32": torch.float32}


def _dtype_name(dt: torch.dtype) -> str:
    return str(dt).replace("torch.", "")


def _pack_json(d: dict) -> torch.Tensor:
    return torch.tensor(list(json.dumps(d).encode("utf-8")), dtype=torch.uint8)


def _unpack_json(t: torch.Tensor) -> dict:
    return json.loads(bytes(t.cpu().to(torch.uint8).tolist()).decode("utf-8"))


def quant_state_tensors(prefix: str, packed: torch.Tensor, qs: QuantState) -> Dict[str, torch.Tensor]:
    """The safetensors entries of one weight (``prefix`` ends in ``.weight``)."""
    if qs.quant_type not in (None, "nf4"):
        raise ValueError("only nf4 quant states are supported")
    out = {prefix: packed.detach().contiguous().cpu(),
           f"{prefix}.absmax": qs.absmax.detach().contiguous().cpu(),
           f"{prefix}.quant_map": qs.code.detach().to(torch.float32).cpu().clone()}
    meta = {"quant_type": "nf4", "blocksize": int(qs.blocksize), "dtype": _dtype_name(qs.dtype),
            "shape": [int(s) for s in qs.shape]}
    if qs.state2 is not None:
        out[f"{prefix}.nested_absmax"] = qs.state2.absmax.detach().to(torch.float32).contiguous().cpu()
        out[f"{prefix}.nested_quant_map"] = qs.state2.code.detach().to(torch.float32).cpu().clone()
        off = qs.offset
        meta.update({"nested_blocksize": int(qs.state2.blocksize), "nested_dtype": _dtype_name(qs.state2.dtype),
                     "nested_offset": float(off.item() if torch.is_tensor(off) else off)})
    out[f"{prefix}.{QS_SUFFIX}"] = _pack_json(meta)
    return out


def save_nf4_safetensors(path: str, weights: Dict[str, Tuple[torch.Tensor, QuantState]]) -> None:
    """Write ``{"<module>.weight": (packed, quant_state), ...}`` as one safetensors file."""
    from safetensors.torch import save_file

    tensors: Dict[str, torch.Tensor] = {}
    for prefix, (packed, qs) in weights.items():
        tensors.update(quant_state_tensors(prefix, packed, qs))
    save_file(tensors, path)


def quant_state_from_tensors(prefix: str, t: Dict[str, torch.Tensor], device) -> QuantState:
    meta = _unpack_json(t[f"{prefix}.{QS_SUFFIX}"])
    if meta.get("quant_type") != "nf4":
        raise ValueError(f"{prefix}: quant_type {meta.get('quant_type')!r} is not nf4")
    state2 = None
    offset = None
    if f"{prefix}.nested_absmax" in t:
        state2 = QuantState(absmax=t[f"{prefix}.nested_absmax"].to(device),
                            code=t[f"{prefix}.nested_quant_map"].to(device),
                            blocksize=int(meta["nested_blocksize"]),
                            dtype=_DT_NAMES[meta.get("nested_dtype", "float32")])
        offset = torch.tensor(float(meta["nested_offset"]), dtype=torch.float32, device=device)
    return QuantState(absmax=t[f"{prefix}.absmax"].to(device), shape=torch.Size(meta["shape"]),
                      code=t[f"{prefix}.quant_map"].to(device), blocksize=int(meta["blocksize"]),
                      quant_type="nf4", dtype=_DT_NAMES[meta["dtype"]], offset=offset, state2=state2)


def load_nf4_safetensors(path: str, device="cpu") -> Dict[str, Linear4bit]:
    """Read every NF4 weight of a safetensors file into ``Linear4bit``-layout modules.

    Keys: ``"<module>"`` (the prefix without ``.weight``) -> module with
    ``weight`` (Params4bit, uint8 packed, ``.quant_state``), ``out_features``,
    ``in_features``.  Non-NF4 tensors in the file are ignored.
    """
    from safetensors import safe_open

    tensors: Dict[str, torch.Tensor] = {}
    with safe_open(path, framework="pt", device="cpu") as f:
        keys = list(f.keys())
        prefixes = [k[: -len(QS_SUFFIX) - 1] for k in keys if k.endswith("." + QS_SUFFIX)]
        # only the NF4 weights' entries are read (a checkpoint's other tensors --
        # embeddings, norms, unquantized heads -- stay on disk)
        wanted = set(prefixes)
        wanted.update(f"{p}.{s}" for p in prefixes for s in
                      ("absmax", "quant_map", "nested_absmax", "nested_quant_map", QS_SUFFIX))
        for k in keys:
            if k in wanted:
                tensors[k] = f.get_tensor(k)
    out: Dict[str, Linear4bit] = {}
    for prefix in sorted(prefixes):
        qs = quant_state_from_tensors(prefix, tensors, device)
        m, n = int(qs.shape[0]), int(qs.shape[1])
        mod = Linear4bit.__new__(Linear4bit)
        torch.nn.Module.__init__(mod)
        mod.in_features, mod.out_features, mod.compute_dtype = n, m, qs.dtype
        mod.weight = Params4bit(tensors[prefix].to(device), qs)
        mod.bias = None
        name = prefix[: -len(".weight")] if prefix.endswith(".weight") else prefix
        out[name] = mod
    return out
