"""msgpack wire format for traced computations.

Bit-compatible with the reference's ``pymoose/pymoose/computation/utils.py:84-175``
(``__type__``-tagged maps; ndarrays as ``{dtype, items, shape}``), so bytes produced by
either front-end can be loaded by the other.
"""
import re
from dataclasses import fields

import msgpack
import numpy as np

from moose_amd.computation import computation as comp_base
from moose_amd.computation import dtypes
from moose_amd.computation import operations as ops
from moose_amd.computation import placements as plc
from moose_amd.computation import types as ty
from moose_amd.computation import values

_TYPE_CLASSES = [
    plc.HostPlacement,
    plc.ReplicatedPlacement,
    plc.MirroredPlacement,
    ty.AesKeyType,
    ty.AesTensorType,
    ty.BytesType,
    ty.FloatType,
    ty.IntType,
    ty.ShapeType,
    ty.StringType,
    ty.TensorType,
    ty.UnitType,
    ty.UnknownType,
    values.FloatConstant,
    values.IntConstant,
    values.ShapeConstant,
    values.StringConstant,
    values.TensorConstant,
    values.BytesConstant,
] + list(ops.OPERATION_CLASSES.values())

TYPE_NAMES = {c.__name__: c for c in _TYPE_CLASSES}
FIXED_DTYPE_REGEX = re.compile(r"fixed([0-9]+)_([0-9]+)")


def serialize_computation(computation):
    return msgpack.packb(computation, default=_encode, use_bin_type=True)


def deserialize_computation(bytes_stream):
    return msgpack.unpackb(
        bytes_stream, object_hook=_decode, raw=False, strict_map_key=False
    )


def _encode(val):
    if isinstance(val, comp_base.Computation):
        return {
            "__type__": "Computation",
            "operations": val.operations,
            "placements": val.placements,
        }
    if isinstance(val, ops.OpSignature):
        return {
            "__type__": "OpSignature",
            "input_types": val.input_types,
            "return_type": val.return_type,
        }
    if isinstance(val, dtypes.DType):
        if FIXED_DTYPE_REGEX.match(val.name):
            return {
                "__type__": "DType",
                "name": "fixed",
                "integral_precision": val.integral_precision,
                "fractional_precision": val.fractional_precision,
            }
        return {"__type__": "DType", "name": val.name}
    if isinstance(val, np.ndarray):
        return {
            "__type__": "ndarray",
            "dtype": str(val.dtype),
            "items": val.flatten().tolist(),
            "shape": list(val.shape),
        }
    if isinstance(val, slice):
        return {
            "__type__": "PySlice",
            "start": val.start,
            "step": val.step,
            "stop": val.stop,
        }
    if isinstance(val, (ops.Operation, ty.ValueType, plc.Placement, values.Value)):
        name = type(val).__name__
        if name not in TYPE_NAMES:
            raise NotImplementedError(name)
        d = {f.name: getattr(val, f.name) for f in fields(val)}
        d["__type__"] = name
        return d
    if isinstance(val, tuple):
        return list(val)
    raise NotImplementedError(f"{type(val)}")


def _decode(obj):
    tname = obj.get("__type__")
    if tname is None:
        return obj
    if tname == "Computation":
        return comp_base.Computation(
            operations=obj["operations"], placements=obj["placements"]
        )
    if tname == "DType":
        name = obj["name"]
        if name == "fixed":
            return dtypes.fixed(obj["integral_precision"], obj["fractional_precision"])
        m = FIXED_DTYPE_REGEX.match(name)
        if m is not None:
            return dtypes.fixed(int(m.group(1)), int(m.group(2)))
        return dtypes.BY_NAME[name]
    if tname == "OpSignature":
        return ops.OpSignature(
            input_types=obj["input_types"], return_type=obj["return_type"]
        )
    if tname == "ndarray":
        return np.array(obj["items"], dtype=obj["dtype"]).reshape(obj["shape"])
    if tname == "PySlice":
        return slice(obj["start"], obj["stop"], obj["step"])
    cls = TYPE_NAMES[tname]
    kwargs = {k: v for k, v in obj.items() if k != "__type__"}
    return cls(**kwargs)
