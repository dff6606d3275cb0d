"""Tensor dtypes of the eDSL (API-compatible with ``pymoose.computation.dtypes``).

Parity: reference ``pymoose/pymoose/computation/dtypes.py:125-258``.  A DType is a
small immutable record; fixed-point dtypes carry ``(integral, fractional)`` bits.
"""
from __future__ import annotations

import numpy as np


class DType:
    __slots__ = ("_name", "_short", "_np", "_flags", "_prec")

    _FLAG_NAMES = (
        "is_native",
        "is_fixedpoint",
        "is_integer",
        "is_float",
        "is_signed",
        "is_boolean",
    )

    def __init__(self, name, short, numpy_dtype, flags, precision=(None, None)):
        self._name = name
        self._short = short
        self._np = numpy_dtype
        self._flags = frozenset(flags)
        self._prec = tuple(precision)

    # flag accessors -------------------------------------------------------
    def _flag(self, f):
        return f in self._flags

    is_native = property(lambda self: self._flag("is_native"))
    is_fixedpoint = property(lambda self: self._flag("is_fixedpoint"))
    is_integer = property(lambda self: self._flag("is_integer"))
    is_float = property(lambda self: self._flag("is_float"))
    is_signed = property(lambda self: self._flag("is_signed"))
    is_boolean = property(lambda self: self._flag("is_boolean"))

    @property
    def integral_precision(self):
        return self._prec[0]

    @property
    def fractional_precision(self):
        return self._prec[1]

    @property
    def name(self):
        return self._name

    @property
    def numpy_dtype(self):
        return self._np

    def __str__(self):
        return self._name

    def __repr__(self):
        return self._short

    def __eq__(self, other):
        return isinstance(other, DType) and (self._name, self._short) == (
            other._name,
            other._short,
        )

    def __hash__(self):
        return hash((self._name, self._short))


_N, _FX, _I, _F, _S, _B = (
    "is_native",
    "is_fixedpoint",
    "is_integer",
    "is_float",
    "is_signed",
    "is_boolean",
)

int32 = DType("int32", "i32", np.int32, {_N, _I, _S})
int64 = DType("int64", "i64", np.int64, {_N, _I, _S})
uint32 = DType("uint32", "u32", np.uint32, {_N, _I})
uint64 = DType("uint64", "u64", np.uint64, {_N, _I})
float32 = DType("float32", "f32", np.float32, {_N, _F, _S})
float64 = DType("float64", "f64", np.float64, {_N, _F, _S})
bool_ = DType("bool_", "bool", np.bool_, {_N, _B})
ring64 = DType("ring64", "ring64", None, {_I})


def fixed(integ, frac):
    """Fixed-point dtype with ``integ`` integral and ``frac`` fractional bits."""
    for p in (integ, frac):
        if not isinstance(p, int):
            raise TypeError("Fixed-point dtype expects integers for its bounds.")
    return DType(
        f"fixed{integ}_{frac}", f"q{integ}.{frac}", None, {_FX, _S}, (integ, frac)
    )


BY_NAME = {
    d.name: d for d in (int32, int64, uint32, uint64, float32, float64, bool_, ring64)
}

__all__ = [
    "bool_",
    "DType",
    "fixed",
    "float32",
    "float64",
    "int32",
    "int64",
    "ring64",
    "uint32",
    "uint64",
]
