"""Pickle-free msgpack codec for argument / result dictionaries crossing process
boundaries (workers, the choreography store, checkpoint files).

numpy arrays travel as ``{"__nd__": dtype-string, "shape": [...], "data": raw bytes}``;
strings, bytes, ints, floats, bools, None, lists and dicts are native msgpack.
"""
from __future__ import annotations

import msgpack
import numpy as np


def _enc(v):
    if isinstance(v, np.ndarray):
        if v.dtype == object:
            raise TypeError("object arrays cannot be encoded")
        a = np.ascontiguousarray(v)
        return {"__nd__": a.dtype.str, "shape": list(a.shape), "data": a.tobytes()}
    if isinstance(v, np.generic):
        return _enc(np.asarray(v))
    if isinstance(v, tuple):
        return {"__tuple__": list(v)}
    try:
        import torch

        if isinstance(v, torch.Tensor):
            return _enc(v.detach().cpu().numpy())
    except ImportError:  # pragma: no cover
        pass
    raise TypeError(f"cannot encode {type(v).__name__}")


def _dec(obj):
    if "__nd__" in obj:
        a = np.frombuffer(obj["data"], dtype=np.dtype(obj["__nd__"]))
        return a.reshape(obj["shape"]).copy()
    if "__tuple__" in obj:
        return tuple(obj["__tuple__"])
    return obj


def dumps(value) -> bytes:
    return msgpack.packb(value, default=_enc, use_bin_type=True, strict_types=True)


def loads(data: bytes):
    return msgpack.unpackb(data, object_hook=_dec, raw=False, strict_map_key=False)
