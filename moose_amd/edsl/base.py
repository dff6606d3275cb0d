"""The Python eDSL: placements, arguments, expressions and op builders.

API-compatible with ``pymoose.edsl.base`` (reference ``pymoose/pymoose/edsl/base.py``,
49 op builders at ``:611-1771``).  Where the reference defines one Expression
dataclass per op, here every expression is a single :class:`Expression` record with an
op ``kind`` and an ``attrs`` dict; the tracer (``tracer.py``) maps kinds to IR
operations through one table.
"""
from __future__ import annotations

import builtins
import functools as ft
import inspect
from dataclasses import dataclass
from dataclasses import field
from typing import Any
from typing import Dict
from typing import List
from typing import Optional

import numpy as np

from moose_amd.computation import dtypes
from moose_amd.computation import types as ty
from moose_amd.computation import values

EllipsisType = type(...)

CURRENT_PLACEMENT: List = []
_CURRENT_RUNTIME = None

_NUMPY_DTYPES_MAP = {
    np.dtype("uint32"): dtypes.uint32,
    np.dtype("uint64"): dtypes.uint64,
    np.dtype("int32"): dtypes.int32,
    np.dtype("int64"): dtypes.int64,
    np.dtype("float32"): dtypes.float32,
    np.dtype("float64"): dtypes.float64,
    np.dtype("bool"): dtypes.bool_,
}


def _np_to_moose_dtype(d):
    try:
        return _NUMPY_DTYPES_MAP.get(np.dtype(d))
    except TypeError:
        return None


def get_current_runtime():
    return _CURRENT_RUNTIME


def set_current_runtime(runtime):
    global _CURRENT_RUNTIME
    _CURRENT_RUNTIME = runtime


# ---------------------------------------------------------------------------
# placements
# ---------------------------------------------------------------------------
@dataclass
class PlacementExpression:
    name: str

    def __enter__(self):
        CURRENT_PLACEMENT.append(self)
        return self

    def __exit__(self, *exc):
        CURRENT_PLACEMENT.pop(-1)

    def __hash__(self):
        return hash(self.name)


@dataclass(eq=True)
class HostPlacementExpression(PlacementExpression):
    def __hash__(self):
        return hash(self.name)


@dataclass(eq=True)
class MirroredPlacementExpression(PlacementExpression):
    players: List[PlacementExpression] = field(default_factory=list)

    def __hash__(self):
        return hash(self.name)


@dataclass(eq=True)
class ReplicatedPlacementExpression(PlacementExpression):
    players: List[PlacementExpression] = field(default_factory=list)

    def __hash__(self):
        return hash(self.name)


def host_placement(name):
    return HostPlacementExpression(name=name)


def mirrored_placement(name, players):
    return MirroredPlacementExpression(name=name, players=list(players))


def replicated_placement(name, players):
    return ReplicatedPlacementExpression(name=name, players=list(players))


def get_current_placement():
    return CURRENT_PLACEMENT[-1]


def _materialize_placement_arg(plc):
    plc = plc or get_current_placement()
    if not isinstance(plc, PlacementExpression):
        raise TypeError(f"Expected value of type Placement, found {type(plc)}.")
    return plc


# ---------------------------------------------------------------------------
# arguments and expressions
# ---------------------------------------------------------------------------
@dataclass(init=False)
class Argument:
    """Type annotation for computation parameters (placement + value type)."""

    placement: PlacementExpression
    dtype: Optional[dtypes.DType] = None
    vtype: Optional[ty.ValueType] = None

    def __init__(self, placement, dtype=None, vtype=None):
        self.placement = placement
        self.dtype = dtype
        self.vtype = _maybe_lift_dtype_to_tensor_vtype(dtype, vtype)


@dataclass(eq=False)
class Expression:
    """One node of the traced expression DAG.

    ``kind`` names the op (``"add"``, ``"dot"``, ``"cast"`` ...); ``attrs`` carries its
    static attributes (``axis``, ``tag`` ...).
    """

    kind: str
    placement: PlacementExpression
    inputs: List["Expression"]
    vtype: Optional[ty.ValueType]
    attrs: Dict[str, Any] = field(default_factory=dict)

    def __hash__(self):
        return id(self)

    def __getattr__(self, item):
        # attribute sugar: expr.axis, expr.tag, expr.arg_name ...
        attrs = self.__dict__.get("attrs")
        if attrs is not None and item in attrs:
            return attrs[item]
        raise AttributeError(item)

    # slicing sugar
    def __getitem__(self, slice_spec):
        if isinstance(self.vtype, (ty.TensorType, ty.AesTensorType)):
            if isinstance(slice_spec, (slice, EllipsisType)):
                slice_spec = (slice_spec,)
            if not isinstance(slice_spec, (list, tuple)):
                raise ValueError("Tensor indexing expects slices or Ellipsis")
            rewritten = []
            for s in slice_spec:
                if isinstance(s, EllipsisType):
                    rewritten.append(slice(None, None, None))
                elif isinstance(s, slice):
                    rewritten.append(s)
                else:
                    raise ValueError(
                        "Indexing with other types different than Ellipsis and slice "
                        "is not yet supported."
                    )
            return strided_slice(self, slices=rewritten)
        if isinstance(self.vtype, ty.ShapeType):
            if isinstance(slice_spec, (tuple, list)):
                if len(slice_spec) != 2:
                    raise ValueError("Indexing ShapeType requires a simple slice.")
                begin, end = slice_spec
            elif isinstance(slice_spec, slice):
                if slice_spec.step is not None:
                    raise ValueError("Indexing ShapeType requires a simple slice.")
                begin, end = slice_spec.start, slice_spec.stop
            else:
                raise ValueError("Indexing ShapeType requires a simple slice.")
            return sliced(self, begin, end)
        raise IndexError(f"Expression of vtype {self.vtype} is not slice-able.")

    # arithmetic sugar
    def __neg__(self):
        _check_arithmetickable(self, "negate")
        if isinstance(self.vtype, ty.TensorType) and not self.vtype.dtype.is_signed:
            raise TypeError(f"Cannot negate Tensor of unsigned DType {self.vtype.dtype}.")
        return mul(constant(-1, vtype=self.vtype), self)

    def __abs__(self):
        _check_arithmetickable(self, "abs")
        if isinstance(self.vtype, ty.TensorType) and not self.vtype.dtype.is_signed:
            return self
        return abs(self)

    def __add__(self, o):
        return _dunder(self, o, add, "add")

    def __radd__(self, o):
        return _dunder(o, self, add, "add")

    def __sub__(self, o):
        return _dunder(self, o, sub, "subtract")

    def __rsub__(self, o):
        return _dunder(o, self, sub, "subtract")

    def __mul__(self, o):
        return _dunder(self, o, mul, "multiply")

    def __rmul__(self, o):
        return _dunder(o, self, mul, "multiply")

    def __truediv__(self, o):
        return _dunder(self, o, div, "divide")

    def __rtruediv__(self, o):
        return _dunder(o, self, div, "divide")

    def __matmul__(self, o):
        return _dunder(self, o, dot, "dot-product")

    def __rmatmul__(self, o):
        return _dunder(o, self, dot, "dot-product")

    def __gt__(self, o):
        return _dunder(self, o, greater, "greater-than")

    def __lt__(self, o):
        return _dunder(self, o, less, "less-than")

    __iadd__ = __add__
    __isub__ = __sub__
    __imul__ = __mul__
    __itruediv__ = __truediv__
    __imatmul__ = __matmul__


def _dunder(x, y, fn, desc):
    _check_arithmetickable(x, desc)
    _check_arithmetickable(y, desc)
    return fn(x, y)


def _check_arithmetickable(expr, fn_name):
    if not isinstance(expr, Expression) or not isinstance(
        expr.vtype, (ty.TensorType, ty.FloatType, ty.IntType)
    ):
        raise TypeError(f"Value of vtype {getattr(expr, 'vtype', expr)} is not {fn_name}-able.")


def _expr(kind, inputs, vtype, placement, **attrs):
    return Expression(
        kind=kind,
        placement=_materialize_placement_arg(placement),
        inputs=list(inputs),
        vtype=vtype,
        attrs=attrs,
    )


# ---------------------------------------------------------------------------
# type helpers
# ---------------------------------------------------------------------------
def _assimilate_arg_vtypes(lhs_vtype, rhs_vtype, fn_name):
    if isinstance(lhs_vtype, ty.TensorType) and isinstance(rhs_vtype, ty.TensorType):
        if lhs_vtype.dtype != rhs_vtype.dtype:
            raise ValueError(
                f"Function `{fn_name}` expected arguments of similar dtype: "
                f"found mismatched dtypes `{lhs_vtype.dtype}` and `{rhs_vtype.dtype}`."
            )
        return lhs_vtype
    if lhs_vtype != rhs_vtype:
        raise ValueError(
            f"Function `{fn_name}` expected arguments of similar type: "
            f"found mismatched types `{lhs_vtype}` and `{rhs_vtype}`."
        )
    return lhs_vtype


def _maybe_lift_dtype_to_tensor_vtype(dtype, vtype):
    if dtype is None:
        return vtype
    if vtype is None:
        return ty.TensorType(dtype)
    if isinstance(vtype, ty.TensorType) and vtype.dtype != dtype:
        raise ValueError(
            f"Inconsistent type information for tensor: dtype {dtype} is "
            f"inconsistent with tensor type {vtype}."
        )
    return vtype


def _check_array_args(arrays, fn):
    if not isinstance(arrays, (tuple, list)):
        raise ValueError(
            f"Inputs to `{fn}` must be array-like, found argument of type {type(arrays)}."
        )
    vt = arrays[0].vtype
    if not isinstance(vt, ty.TensorType):
        raise ValueError(f"Inputs must be have vtype TensorType, found {vt}.")
    for a in arrays:
        if not isinstance(a.vtype, ty.TensorType) or a.vtype.dtype != vt.dtype:
            raise ValueError(
                f"Values passed to {fn} must be same dtype: found {a.vtype} and {vt}."
            )
    return vt


def _shape_operand(shape, placement):
    """Lift a python list/tuple shape into a host-placed ShapeConstant."""
    if isinstance(shape, (list, tuple)):
        plc = _materialize_placement_arg(placement)
        host = plc.players[0] if isinstance(plc, ReplicatedPlacementExpression) else plc
        return constant(values.ShapeConstant(value=tuple(shape)), vtype=ty.ShapeType(),
                        placement=host)
    assert isinstance(shape, Expression)
    return shape


# ---------------------------------------------------------------------------
# op builders
# ---------------------------------------------------------------------------
def add_n(arrays, placement=None):
    """Elementwise sum of a list of tensors."""
    vt = _check_array_args(arrays, "add_n")
    return _expr("add_n", arrays, vt, placement)


def identity(x, placement=None):
    """Identity; may move ``x`` to another placement."""
    return _expr("identity", [x], x.vtype, placement)


def concatenate(arrays, axis=0, placement=None):
    """Concatenate tensors along an existing ``axis``."""
    vt = _check_array_args(arrays, "concatenate")
    return _expr("concatenate", arrays, vt, placement, axis=axis)


def maximum(arrays, placement=None):
    """Elementwise maximum of a list of tensors."""
    vt = _check_array_args(arrays, "maximum")
    return _expr("maximum", arrays, vt, placement)


def decrypt(key, ciphertext, placement=None):
    """AES-GCM decrypt ``ciphertext`` (AesTensorType) with ``key`` (AesKeyType)."""
    if not isinstance(key.vtype, ty.AesKeyType):
        raise ValueError(f"Parameter `key` expected to be of type AesKeyType, found {key.vtype}.")
    if not isinstance(ciphertext.vtype, ty.AesTensorType):
        raise ValueError(
            f"Parameter `ciphertext` expected to be of type AesTensorType, found {ciphertext.vtype}."
        )
    return _expr("decrypt", [key, ciphertext], ty.TensorType(ciphertext.vtype.dtype),
                 placement)


def constant(value, dtype=None, vtype=None, placement=None):
    """Embed a constant (python scalar, string, ndarray or Shape/other Constant)."""
    placement = _materialize_placement_arg(placement)
    vtype = _maybe_lift_dtype_to_tensor_vtype(dtype, vtype)
    if isinstance(value, np.ndarray):
        moose_dtype = _np_to_moose_dtype(value.dtype)
        if moose_dtype is None:
            raise NotImplementedError(
                f"Tensors of dtype `{value.dtype}` not supported as graph constants."
            )
        if vtype is not None and moose_dtype != vtype.dtype:
            target = dtype or vtype.dtype
            inner = constant(value, dtype=moose_dtype, placement=placement)
            return cast(inner, target, placement)
        vtype = vtype or ty.TensorType(moose_dtype)
        value = values.TensorConstant(value=value)
    elif isinstance(value, bool):
        value = values.TensorConstant(value=np.array(value))
        vtype = vtype or ty.TensorType(dtypes.bool_)
    elif isinstance(value, (float, int)):
        if isinstance(vtype, ty.TensorType) and vtype.dtype.is_fixedpoint:
            return constant(np.array(value), vtype=vtype, placement=placement)
        fallback = ty.FloatType() if isinstance(value, float) else ty.IntType()
        value, vtype = _interpret_numeric_value(value, vtype, fallback)
    elif isinstance(value, str):
        vtype = vtype or ty.StringType()
        if not isinstance(vtype, ty.StringType):
            raise ValueError(
                f"Constant value of type `str` does not match user-supplied vtype `{vtype}`."
            )
        value = values.StringConstant(value=value)
    return Expression("constant", placement, [], vtype, {"value": value})


def _interpret_numeric_value(value, vtype, fallback_vtype):
    vtype = vtype or fallback_vtype
    if isinstance(vtype, ty.TensorType):
        d = vtype.dtype
        if not d.is_float and not d.is_integer:
            raise TypeError(f"Cannot interpret scalar constant as dtype {d}.")
        return values.TensorConstant(np.array(value, dtype=d.numpy_dtype)), vtype
    if isinstance(vtype, ty.FloatType):
        return values.FloatConstant(value), vtype
    if isinstance(vtype, ty.IntType):
        return values.IntConstant(value), vtype
    raise TypeError(f"Cannot interpret numeric constant as non-numeric type {vtype}.")


def _binary(kind, lhs, rhs, placement, vtype=None):
    assert isinstance(lhs, Expression) and isinstance(rhs, Expression)
    if vtype is None:
        vtype = _assimilate_arg_vtypes(lhs.vtype, rhs.vtype, kind)
    return _expr(kind, [lhs, rhs], vtype, placement)


def add(lhs, rhs, placement=None):
    """``lhs + rhs`` (elementwise)."""
    return _binary("add", lhs, rhs, placement)


def sub(lhs, rhs, placement=None):
    """``lhs - rhs`` (elementwise)."""
    return _binary("sub", lhs, rhs, placement)


def mul(lhs, rhs, placement=None):
    """``lhs * rhs`` (elementwise)."""
    return _binary("mul", lhs, rhs, placement)


def dot(lhs, rhs, placement=None):
    """Tensor contraction (``np.dot`` semantics for rank 1/2)."""
    return _binary("dot", lhs, rhs, placement)


def div(lhs, rhs, placement=None):
    """``lhs / rhs`` (elementwise)."""
    return _binary("div", lhs, rhs, placement)


def less(lhs, rhs, placement=None):
    """``lhs < rhs`` -> bool tensor."""
    return _binary("less", lhs, rhs, placement, vtype=ty.TensorType(dtypes.bool_))


def greater(lhs, rhs, placement=None):
    """``lhs > rhs`` -> bool tensor."""
    return _binary("greater", lhs, rhs, placement, vtype=ty.TensorType(dtypes.bool_))


def logical_and(lhs, rhs, placement=None):
    """Boolean AND."""
    return _binary("and", lhs, rhs, placement)


def logical_or(lhs, rhs, placement=None):
    """Boolean OR."""
    return _binary("or", lhs, rhs, placement)


def inverse(x, placement=None):
    """Float matrix inverse (host only)."""
    if not isinstance(x.vtype, ty.TensorType):
        raise ValueError("`inverse` operation only supports arguments of type TensorType.")
    if x.vtype.dtype not in (dtypes.float32, dtypes.float64):
        raise ValueError("`inverse` operation only supports `float32` or `float64`.")
    return _expr("inverse", [x], x.vtype, placement)


def expand_dims(x, axis, placement=None):
    """Insert singleton dimension(s) at ``axis``."""
    if isinstance(axis, int):
        axis = [axis]
    elif isinstance(axis, (tuple, list)):
        for a in axis:
            if not isinstance(a, int):
                raise ValueError(f"`axis` argument must be int or list of ints, found {type(a)}")
        axis = list(axis)
    return _expr("expand_dims", [x], x.vtype, placement, axis=axis)


def squeeze(x, axis=None, placement=None):
    """Drop singleton dimensions."""
    return _expr("squeeze", [x], x.vtype, placement, axis=axis)


def ones(shape, dtype, placement=None):
    """Tensor of ones of the given shape."""
    return _expr("ones", [_shape_operand(shape, placement)], ty.TensorType(dtype), placement)


def zeros(shape, dtype, placement=None):
    """Tensor of zeros of the given shape."""
    return _expr("zeros", [_shape_operand(shape, placement)], ty.TensorType(dtype), placement)


def square(x, placement=None):
    """``x * x``."""
    return mul(x, x, placement=placement)


def sum(x, axis=None, placement=None):
    """Sum-reduce along ``axis`` (all axes if None)."""
    return _expr("sum", [x], x.vtype, placement, axis=axis)


def mean(x, axis=None, placement=None):
    """Mean-reduce along ``axis`` (all axes if None)."""
    return _expr("mean", [x], x.vtype, placement, axis=axis)


def _unary(kind):
    def builder(x, placement=None):
        assert isinstance(x, Expression)
        return _expr(kind, [x], x.vtype, placement)

    builder.__name__ = kind
    builder.__doc__ = f"Elementwise ``{kind}``."
    return builder


exp = _unary("exp")
sqrt = _unary("sqrt")
sigmoid = _unary("sigmoid")
relu = _unary("relu")
log = _unary("log")
log2 = _unary("log2")
abs = _unary("abs")
transpose = _unary("transpose")


def softmax(x, axis, upmost_index, placement=None):
    """Softmax along ``axis`` over the first ``upmost_index`` entries."""
    return _expr("softmax", [x], x.vtype, placement, axis=axis, upmost_index=upmost_index)


def argmax(x, axis, upmost_index, placement=None):
    """Index of the maximum along ``axis``."""
    return _expr("argmax", [x], x.vtype, placement, axis=axis, upmost_index=upmost_index)


def shape(x, placement=None):
    """Shape of a tensor."""
    return _expr("shape", [x], ty.ShapeType(), placement)


def index_axis(x, axis, index, placement=None):
    """``x`` indexed at ``index`` along ``axis`` (drops the axis)."""
    if not isinstance(axis, int) or axis < 0:
        raise ValueError(f"`axis` argument must be int greater or equal to 0, found {axis}")
    if not isinstance(index, int) or index < 0:
        raise ValueError(f"`index` argument must be int greater or equal to 0, found {index}")
    return _expr("index_axis", [x], x.vtype, placement, axis=axis, index=index)


def select(x, axis, index, placement=None):
    """Keep entries along ``axis`` where the boolean ``index`` is 1."""
    if not isinstance(axis, int):
        raise ValueError(f"`axis` argument must be int, found {type(axis)}")
    return _expr("select", [x, index], x.vtype, placement, axis=axis)


def sliced(x, begin, end, placement=None):
    """``x[begin:end]`` along the first axis (tensors) or of a shape."""
    assert isinstance(begin, int) and isinstance(end, int)
    return _expr("slice", [x], x.vtype, placement, begin=begin, end=end)


def strided_slice(x, slices, placement=None):
    """General python-slice indexing."""
    for s in slices:
        if not isinstance(s, slice):
            raise ValueError(f"`slices` argument must a list/tuple of slices, found {type(s)}")
    return _expr("strided_slice", [x], x.vtype, placement, slices=list(slices))


def atleast_2d(x, to_column_vector=False, placement=None):
    """Promote rank<2 tensors to rank 2."""
    return _expr("atleast_2d", [x], x.vtype, placement, to_column_vector=to_column_vector)


def reshape(x, shape, placement=None):
    """Reshape ``x`` to ``shape`` (list/tuple or Shape expression)."""
    return _expr("reshape", [x, _shape_operand(shape, placement)], x.vtype, placement)


def mux(selector, x, y, placement=None):
    """``selector ? x : y`` on a replicated placement."""
    assert isinstance(selector.vtype, ty.TensorType) and selector.vtype.dtype.is_boolean
    assert isinstance(x.vtype, ty.TensorType) and x.vtype.dtype.is_fixedpoint
    assert isinstance(y.vtype, ty.TensorType) and y.vtype.dtype.is_fixedpoint
    plc = _materialize_placement_arg(placement)
    assert isinstance(plc, ReplicatedPlacementExpression)
    vt = _assimilate_arg_vtypes(x.vtype, y.vtype, "mux")
    return _expr("mux", [selector, x, y], vt, plc)


def cast(x, dtype, placement=None):
    """Convert a tensor to ``dtype`` (float<->fixed encode/decode, int casts...)."""
    if not isinstance(x.vtype, ty.TensorType):
        raise ValueError(f"Argument to `cast` operation must be tensor, found {x.vtype}.")
    if x.vtype.dtype is None:
        raise ValueError("Argument to `cast` function must have well-defined dtype.")
    if dtype is None:
        raise ValueError("Invalid `dtype` argument to `cast` function: cannot cast to None.")
    if isinstance(dtype, dtypes.DType):
        target = dtype
    else:
        target = _np_to_moose_dtype(dtype)
        if target is None:
            raise ValueError(f"Unsupported dtype arg in `cast` function: {dtype}.")
    if x.vtype.dtype == target:
        return x
    return _expr("cast", [x], ty.TensorType(target), placement)


def _string_operand(v, placement, fn, what):
    if isinstance(v, str):
        return constant(v, placement=placement, vtype=ty.StringType())
    if isinstance(v, Argument) and v.vtype not in (ty.StringType(), None):
        raise ValueError(f"Function 'edsl.{fn}' encountered `{what}` of vtype {v.vtype}.")
    if not isinstance(v, Expression):
        raise ValueError(f"Function 'edsl.{fn}' encountered `{what}` of type {type(v)}.")
    return v


def load(key, query="", dtype=None, vtype=None, placement=None):
    """Load a value from the placement's storage."""
    placement = _materialize_placement_arg(placement)
    vtype = _maybe_lift_dtype_to_tensor_vtype(dtype, vtype)
    key = _string_operand(key, placement, "load", "key")
    query = _string_operand(query, placement, "load", "query")
    return _expr("load", [key, query], vtype, placement)


def save(key, value, placement=None):
    """Save ``value`` under ``key`` in the placement's storage."""
    assert isinstance(value, Expression)
    placement = _materialize_placement_arg(placement)
    key = _string_operand(key, placement, "save", "key")
    return _expr("save", [key, value], None, placement)


def output(tag, value, placement=None):
    """Tag an output of the computation."""
    assert isinstance(value, Expression) and isinstance(tag, str)
    return _expr("output", [value], value.vtype, placement, tag=tag)


# ---------------------------------------------------------------------------
# computations
# ---------------------------------------------------------------------------
def computation(func=None, role_map=None):
    """Decorate a python function as an (abstract) Moose computation."""
    if func is None:
        return ft.partial(computation, role_map=role_map)
    return AbstractComputation(func, role_map)


class AbstractComputation:
    def __init__(self, func, role_map):
        if not callable(func):
            raise TypeError(f"Argument `func` should be a callable, but found {type(func)}.")
        if role_map is not None and not isinstance(role_map, dict):
            raise TypeError(
                f"Argument `role_map` should be map of placement names, found {type(role_map)}."
            )
        self.func = func
        self.role_map = role_map

    def __call__(self, *args, **kwargs):
        names = list(inspect.signature(self.func).parameters)
        if len(args) > len(names):
            raise ValueError(f"Too many arguments for `{self.func.__name__}`")
        arguments = dict(zip(names, args))
        for k, v in kwargs.items():
            if k in arguments:
                raise ValueError(f"Argument `{k}` given more than once to `{self.func.__name__}`")
            if k not in names:
                raise ValueError(f"Argument `{k}` is not used by `{self.func.__name__}`")
            arguments[k] = v
        for n in names:
            if n not in arguments:
                raise ValueError(f"Missing argument `{n}` in call to `{self.func.__name__}`")
        runtime = get_current_runtime()
        if not runtime:
            raise RuntimeError("No default runtime found")
        return runtime.evaluate_computation(self, arguments)

    def with_role_map(self, role_map):
        return self.__class__(self.func, role_map)


__all__ = [n for n in dir() if not n.startswith("_") and n not in ("builtins",)]
