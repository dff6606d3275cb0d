"""Convert an eDSL (pymoose-format) computation into the native IR.

Parity: reference ``pymoose/src/computation.rs`` (``PyComputation`` -> ``Computation``,
type map ``:679-699``, placement map ``:555-588``).  As in the reference every
``fixed(i, f)`` becomes ``Fixed128(i, f)`` unless ``fixedpoint_ring=64`` is requested
(then ``Fixed64(i, f)``, the Z_2^64 fast path).
"""
from __future__ import annotations

import numpy as np

from moose_amd.computation import computation as ecomp
from moose_amd.computation import dtypes as edt
from moose_amd.computation import placements as eplc
from moose_amd.computation import types as ety
from moose_amd.computation import values as evals
from moose_amd.ir import types as T
from moose_amd.ir.computation import Computation
from moose_amd.ir.computation import Constant
from moose_amd.ir.computation import HostPlacement
from moose_amd.ir.computation import Mirrored3Placement
from moose_amd.ir.computation import Operation
from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ir.computation import Signature

# eDSL operation class -> (IR kind, operand names | "array", attribute mapper)
_OPS = {
    "AbsOperation": ("Abs", ["x"], None),
    "AddNOperation": ("AddN", "array", None),
    "AddOperation": ("Add", ["lhs", "rhs"], None),
    "ArgmaxOperation": ("Argmax", ["x"], lambda o: {"axis": o.axis, "upmost_index": o.upmost_index}),
    "AtLeast2DOperation": ("AtLeast2D", ["x"], lambda o: {"to_column_vector": bool(o.to_column_vector)}),
    "BitwiseAndOperation": ("And", ["lhs", "rhs"], None),
    "BitwiseOrOperation": ("Or", ["lhs", "rhs"], None),
    "CastOperation": ("Cast", ["x"], None),
    "ConcatenateOperation": ("Concat", "array", lambda o: {"axis": o.axis or 0}),
    "ConstantOperation": ("Constant", [], None),
    "DecryptOperation": ("Decrypt", ["key", "ciphertext"], None),
    "DivOperation": ("Div", ["lhs", "rhs"], None),
    "DotOperation": ("Dot", ["lhs", "rhs"], None),
    "ExpandDimsOperation": ("ExpandDims", ["x"], lambda o: {"axis": list(o.axis)}),
    "ExpOperation": ("Exp", ["x"], None),
    "GreaterOperation": ("Greater", ["lhs", "rhs"], None),
    "IdentityOperation": ("Identity", ["x"], None),
    "IndexAxisOperation": ("IndexAxis", ["x"], lambda o: {"axis": o.axis, "index": o.index}),
    "InputOperation": ("Input", [], lambda o: {"arg_name": o.name}),
    "InverseOperation": ("Inverse", ["x"], None),
    "LessOperation": ("Less", ["lhs", "rhs"], None),
    "LoadOperation": ("Load", ["key", "query"], None),
    "LogOperation": ("Log", ["x"], None),
    "Log2Operation": ("Log2", ["x"], None),
    "MaximumOperation": ("Maximum", "array", None),
    "MeanOperation": ("Mean", ["x"], lambda o: {"axis": o.axis}),
    "MulOperation": ("Mul", ["lhs", "rhs"], None),
    "MuxOperation": ("Mux", ["selector", "x", "y"], None),
    "OnesOperation": ("Ones", ["shape"], None),
    "ZerosOperation": ("Zeros", ["shape"], None),
    "OutputOperation": ("Output", ["value"], lambda o: {"tag": o.tag}),
    "SigmoidOperation": ("Sigmoid", ["x"], None),
    "ReluOperation": ("Relu", ["x"], None),
    "SelectOperation": ("Select", ["index", "x"], lambda o: {"axis": o.axis}),
    "SoftmaxOperation": ("Softmax", ["x"], lambda o: {"axis": o.axis, "upmost_index": o.upmost_index}),
    "ReshapeOperation": ("Reshape", ["x", "shape"], None),
    "SaveOperation": ("Save", ["key", "value"], None),
    "ShapeOperation": ("Shape", ["x"], None),
    "SliceOperation": ("Slice", ["x"], lambda o: {"slice": [(o.begin, o.end, None)]}),
    "StridedSliceOperation": (
        "Slice",
        ["x"],
        lambda o: {"slice": [(s.start if s.start is not None else 0, s.stop, s.step) for s in o.slices]},
    ),
    "SqueezeOperation": ("Squeeze", ["x"], lambda o: {"axis": o.axis}),
    "SqrtOperation": ("Sqrt", ["x"], None),
    "SubOperation": ("Sub", ["lhs", "rhs"], None),
    "SumOperation": ("Sum", ["x"], lambda o: {"axis": o.axis}),
    "TransposeOperation": ("Transpose", ["x"], None),
}

_NP_CONST = {
    np.dtype("float32"): "HostFloat32Tensor",
    np.dtype("float64"): "HostFloat64Tensor",
    np.dtype("int8"): "HostInt8Tensor",
    np.dtype("int16"): "HostInt16Tensor",
    np.dtype("int32"): "HostInt32Tensor",
    np.dtype("int64"): "HostInt64Tensor",
    np.dtype("uint8"): "HostUint8Tensor",
    np.dtype("uint16"): "HostUint16Tensor",
    np.dtype("uint32"): "HostUint32Tensor",
    np.dtype("uint64"): "HostUint64Tensor",
    np.dtype("bool"): "HostBitTensor",
}


def map_dtype(d: edt.DType, fixedpoint_ring=128) -> T.TensorDType:
    if d.is_fixedpoint:
        kind = "Fixed64" if fixedpoint_ring == 64 else "Fixed128"
        return T.TensorDType(kind, d.integral_precision, d.fractional_precision)
    m = {
        "float32": T.FLOAT32,
        "float64": T.FLOAT64,
        "bool_": T.BOOL,
        "uint64": T.UINT64,
        "int64": T.UINT64,
        "int32": T.UINT64,
        "uint32": T.UINT64,
    }
    if d.name not in m:
        raise ValueError(f"unsupported dtype {d}")
    return m[d.name]


def map_type(vt, plc, fixedpoint_ring=128) -> T.Ty:
    if vt is None or isinstance(vt, ety.UnknownType):
        return T.UNKNOWN
    if isinstance(vt, ety.TensorType):
        return T.tensor(map_dtype(vt.dtype, fixedpoint_ring))
    if isinstance(vt, ety.ShapeType):
        kind = "Replicated" if isinstance(plc, ReplicatedPlacement) else "Host"
        return T.Ty("Shape", kind)
    if isinstance(vt, ety.UnitType):
        return T.HOST_UNIT
    if isinstance(vt, ety.StringType):
        return T.HOST_STRING
    if isinstance(vt, ety.AesTensorType):
        return T.Ty("AesTensor")
    if isinstance(vt, ety.AesKeyType):
        return T.Ty("AesKey")
    if isinstance(vt, (ety.FloatType, ety.IntType)):
        return T.Ty("Float64")
    if isinstance(vt, ety.BytesType):
        return T.Ty("HostString")
    raise ValueError(f"unsupported value type {vt}")


def map_constant(v) -> Constant:
    if isinstance(v, evals.TensorConstant):
        arr = np.asarray(v.value)
        kind = _NP_CONST.get(arr.dtype)
        if kind is None:
            raise ValueError(f"unsupported constant dtype {arr.dtype}")
        if kind == "HostBitTensor":
            arr = arr.astype(np.uint8)
        return Constant(kind, arr)
    if isinstance(v, evals.StringConstant):
        return Constant("HostString", v.value)
    if isinstance(v, evals.ShapeConstant):
        return Constant("HostShape", tuple(int(x) for x in v.value))
    if isinstance(v, evals.FloatConstant):
        return Constant("Float64", float(v.value))
    if isinstance(v, evals.IntConstant):
        return Constant("Float64", float(v.value))
    if isinstance(v, evals.BytesConstant):
        return Constant("HostString", v.value.decode("latin-1"))
    raise ValueError(f"unsupported constant {v}")


def convert(comp: ecomp.Computation, fixedpoint_ring=128) -> Computation:
    plcs = {}
    for name, p in comp.placements.items():
        if isinstance(p, eplc.HostPlacement):
            plcs[name] = HostPlacement(p.name)
        elif isinstance(p, eplc.ReplicatedPlacement):
            plcs[name] = ReplicatedPlacement(tuple(p.player_names))
        elif isinstance(p, eplc.MirroredPlacement):
            plcs[name] = Mirrored3Placement(tuple(p.player_names))
        else:
            raise ValueError(f"unsupported placement {p}")
    out = []
    for op in comp.operations.values():
        cls = type(op).__name__
        if cls not in _OPS:
            raise ValueError(f"unsupported eDSL operation {cls}")
        kind, operands, attr_fn = _OPS[cls]
        plc = plcs[op.placement_name]
        if operands == "array":
            names = sorted(op.inputs, key=lambda k: int(k[5:]))
            inputs = [op.inputs[k] for k in names]
            arg_tys = [map_type(op.signature.input_types[names[0]], plc, fixedpoint_ring)]
            variadic = True
        else:
            inputs = [op.inputs[k] for k in operands]
            arg_tys = [map_type(op.signature.input_types.get(k), plc, fixedpoint_ring)
                       for k in operands]
            variadic = False
        ret = map_type(op.signature.return_type, plc, fixedpoint_ring)
        attrs = attr_fn(op) if attr_fn else {}
        if kind == "Constant":
            attrs = {"value": map_constant(op.value)}
        sig = Signature(tuple(arg_tys), ret, variadic)
        out.append(Operation(op.name, kind, inputs, plc, sig, attrs))
    return Computation(out).toposorted()
