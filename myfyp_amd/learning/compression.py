"""Wire compression of model payloads (the FYP MLP's ``model_build_fn(..., compression=)``).

The FYP script builds its model as ``LightningModel(MLP(...), compression=compression)``
(``/root/reference/mlp_pytorch.txt:148-151``): a newer upstream p2pfl compresses the weights a peer
sends. This reference tree has no implementation (its ``LightningModel`` takes no such argument), so
the format here is our own and parity is unpinned; the uncompressed wire format is untouched
(``pickle({"params", "additional_info"})``, ``p2pfl_model.py:81-85``), so peers that do not compress
interoperate with the reference exactly.

``compression`` is a dict of techniques, applied in this order on encode and reversed on decode:

* ``{"topk": {"k": 0.1}}`` — keep the largest-magnitude fraction ``k`` of every floating tensor
  (indices + values; the rest decode as zero). Lossy.
* ``{"ptq": {"dtype": "float16" | "bfloat16" | "int8"}}`` — post-training quantisation of floating
  tensors for transport (int8: symmetric per-tensor scale). Lossy; the model itself stays fp32.
* ``{"zlib": {"level": 6}}`` — lossless deflate of the whole pickled payload.

A compressed payload is ``MAGIC + zlib(pickle(...))`` when zlib is on, else a plain pickle whose
dict carries a ``"compression"`` key; the decoder recognises both and the plain reference format.
Every structure is numpy arrays, ints, floats, strings and plain containers, so the restricted
unpickler (``p2pfl_model.safe_loads``) still decodes it.
"""

from __future__ import annotations

import zlib
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

MAGIC = b"MYFYPZ1\x00"
TECHNIQUES = ("topk", "ptq", "zlib")


def validate(compression: Optional[Dict[str, Any]]) -> Optional[Dict[str, Dict[str, Any]]]:
    if not compression:
        return None
    if not isinstance(compression, dict):
        raise ValueError(f"compression must be a dict of techniques, got {type(compression).__name__}")
    out: Dict[str, Dict[str, Any]] = {}
    for name, opts in compression.items():
        if name not in TECHNIQUES:
            raise ValueError(f"unknown compression technique {name!r} (known: {', '.join(TECHNIQUES)})")
        out[name] = dict(opts or {})
    if "topk" in out:
        k = float(out["topk"].get("k", 0.1))
        if not 0.0 < k <= 1.0:
            raise ValueError("topk.k must be in (0, 1]")
        out["topk"]["k"] = k
    if "ptq" in out:
        dt = out["ptq"].setdefault("dtype", "float16")
        if dt not in ("float16", "bfloat16", "int8"):
            raise ValueError(f"ptq.dtype must be float16, bfloat16 or int8, got {dt!r}")
    return out


def _bf16_bits(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)  # round to nearest even


def _encode_array(a: np.ndarray, c: Dict[str, Dict[str, Any]]) -> Any:
    a = np.asarray(a)
    if not np.issubdtype(a.dtype, np.floating):
        return {"raw": a}
    enc: Dict[str, Any] = {"shape": np.asarray(a.shape, dtype=np.int64), "dtype": str(a.dtype)}
    flat = a.reshape(-1).astype(np.float32)
    if "topk" in c:
        keep = max(1, int(round(c["topk"]["k"] * flat.size)))
        idx = np.argpartition(np.abs(flat), flat.size - keep)[flat.size - keep:] if keep < flat.size else np.arange(flat.size)
        idx = np.sort(idx).astype(np.int64 if flat.size > 2**31 - 1 else np.int32)
        enc["idx"] = idx
        flat = flat[idx]
    if "ptq" in c:
        dt = c["ptq"]["dtype"]
        if dt == "float16":
            enc["q"] = flat.astype(np.float16)
        elif dt == "bfloat16":
            enc["q"] = _bf16_bits(flat)
        else:
            scale = float(np.max(np.abs(flat))) / 127.0 if flat.size else 0.0
            enc["scale"] = scale
            enc["q"] = np.clip(np.rint(flat / scale), -127, 127).astype(np.int8) if scale > 0 else np.zeros(flat.size, np.int8)
        enc["qtype"] = dt
    else:
        enc["v"] = flat
    return enc


# Bounds on peer-supplied payloads: a compressed payload must not be able to make the
# receiver allocate more than this (a zlib bomb, or a tiny top-k payload naming a huge shape). With
# the receiving model's shapes known, the bound is the model's own size.
MAX_DECODED_BYTES = 1 << 30
MAX_ELEMENTS = 1 << 28


def _decode_array(enc: Any, expect: Optional[tuple] = None, max_elems: int = MAX_ELEMENTS) -> np.ndarray:
    if "raw" in enc:
        return np.asarray(enc["raw"])
    shape = tuple(int(s) for s in enc["shape"])
    if any(d < 0 for d in shape):
        raise ValueError(f"compressed tensor: negative dimension in {shape}")
    if expect is not None and tuple(expect) != shape:
        raise ValueError(f"compressed tensor of shape {shape}, the model expects {tuple(expect)}")
    n_elems = int(np.prod(shape, dtype=np.int64)) if shape else 1
    if n_elems > max_elems:
        raise ValueError(f"compressed tensor of {n_elems} elements exceeds the bound {max_elems}")
    if "q" in enc:
        qt = enc["qtype"]
        q = np.asarray(enc["q"])
        if qt == "float16":
            vals = q.astype(np.float32)
        elif qt == "bfloat16":
            vals = (q.astype(np.uint32) << 16).view(np.float32)
        else:
            vals = q.astype(np.float32) * np.float32(enc["scale"])
    else:
        vals = np.asarray(enc["v"], dtype=np.float32)
    n = n_elems
    if "idx" in enc:
        idx = np.asarray(enc["idx"])
        if idx.ndim != 1 or not np.issubdtype(idx.dtype, np.integer) or idx.size != vals.size:
            raise ValueError("compressed tensor: top-k indices must be a 1-D integer array, one per value")
        if idx.size and (idx[0] < 0 or idx[-1] >= n or np.any(np.diff(idx) <= 0)):
            raise ValueError("compressed tensor: top-k indices out of range or not strictly increasing")
        flat = np.zeros(n, dtype=np.float32)
        flat[idx] = vals
    else:
        if vals.size != n:
            raise ValueError(f"compressed tensor: {vals.size} values for shape {shape}")
        flat = vals
    return flat.reshape(shape).astype(np.dtype(enc["dtype"]))


def encode(params: List[np.ndarray], additional_info: Dict[str, Any], compression: Optional[Dict[str, Dict[str, Any]]]) -> bytes:
    """Payload bytes of ``params`` + ``additional_info`` under ``compression`` (None: reference format)."""
    import pickle

    if not compression:
        return pickle.dumps({"params": params, "additional_info": additional_info})
    body = {"params": [_encode_array(p, compression) for p in params], "additional_info": additional_info,
            "compression": sorted(compression)}
    raw = pickle.dumps(body)
    if "zlib" in compression:
        return MAGIC + zlib.compress(raw, int(compression["zlib"].get("level", 6)))
    return raw


def decode(data: bytes, loads, expected_shapes: Optional[List[tuple]] = None) -> Tuple[List[np.ndarray], Dict[str, Any]]:
    """(params, additional_info) of a payload in the reference format or a compressed one; ``loads``
    is the restricted unpickler. ``expected_shapes`` (the receiving model's) bounds what a
    compressed payload may decode to: its inflated size, each tensor's shape, and the top-k
    indices are checked before anything is allocated."""
    max_bytes, max_elems = MAX_DECODED_BYTES, MAX_ELEMENTS
    if expected_shapes:
        model_elems = sum(int(np.prod(s, dtype=np.int64)) if len(s) else 1 for s in expected_shapes)
        max_elems = max(1, model_elems)
        # the pickled payload of an uncompressed fp32 model plus generous framing
        max_bytes = min(MAX_DECODED_BYTES, 8 * model_elems + (16 << 20))
    if data[: len(MAGIC)] == MAGIC:
        d = zlib.decompressobj()
        out = d.decompress(data[len(MAGIC):], max_bytes)
        if d.unconsumed_tail or not d.eof:
            raise ValueError(f"compressed payload inflates past {max_bytes} bytes (or is truncated)")
        data = out
    loaded = loads(data)
    if "compression" in loaded:
        encs = loaded["params"]
        if expected_shapes is not None and len(encs) != len(expected_shapes):
            raise ValueError(f"compressed payload has {len(encs)} tensors, the model {len(expected_shapes)}")
        return [_decode_array(e, None if expected_shapes is None else expected_shapes[i], max_elems) for i, e in enumerate(encs)], loaded["additional_info"]
    return loaded["params"], loaded["additional_info"]
