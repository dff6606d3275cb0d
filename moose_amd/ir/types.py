"""Type system of the native IR: ``Ty`` and ``TensorDType``.

Parity: reference ``moose/src/computation.rs:330-591`` (``values!`` macro, ~62 ``Ty``
variants) and ``moose/src/logical/mod.rs:17-43`` (``TensorDType``/``TensorShape``).
Types are immutable (name, inner) records; the textual form is ``Name`` or
``Name<Inner>`` exactly as the reference prints it.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Optional
from typing import Union


@dataclass(frozen=True)
class TensorDType:
    """Logical tensor element type: Fixed64/Fixed128 carry (integral, fractional)."""

    kind: str  # Fixed64 | Fixed128 | Float32 | Float64 | Bool | Uint64 | Unknown
    integral_precision: int = 0
    fractional_precision: int = 0

    @property
    def is_fixed(self):
        return self.kind in ("Fixed64", "Fixed128")

    @property
    def ring_bits(self):
        return {"Fixed64": 64, "Fixed128": 128}.get(self.kind)

    def to_textual(self):
        if self.is_fixed:
            return f"{self.kind}({self.integral_precision}, {self.fractional_precision})"
        return self.kind

    @staticmethod
    def from_textual(s: str) -> "TensorDType":
        s = s.strip()
        m = re.fullmatch(r"(Fixed64|Fixed128)\(\s*(\d+)\s*,\s*(\d+)\s*\)", s)
        if m:
            return TensorDType(m.group(1), int(m.group(2)), int(m.group(3)))
        if s in ("Float32", "Float64", "Bool", "Uint64", "Unknown"):
            return TensorDType(s)
        raise ValueError(f"unknown TensorDType {s!r}")

    def __str__(self):
        return self.to_textual()


FLOAT32 = TensorDType("Float32")
FLOAT64 = TensorDType("Float64")
BOOL = TensorDType("Bool")
UINT64 = TensorDType("Uint64")
UNKNOWN_DTYPE = TensorDType("Unknown")


def fixed64(i, f):
    return TensorDType("Fixed64", i, f)


def fixed128(i, f):
    return TensorDType("Fixed128", i, f)


SHAPE_KINDS = ("Host", "Replicated", "Additive", "Mirrored", "Unknown")

# All concrete type names of the reference (computation.rs:538-591) plus the
# scalar pseudo-types.  ``Tensor`` and ``Shape`` take an inner parameter.
TYPE_NAMES = [
    "Unknown",
    "HostUnit",
    "HostShape",
    "HostSeed",
    "HostPrfKey",
    "HostString",
    "Shape",
    "Tensor",
    "HostBitTensor",
    "HostBitArray64",
    "HostBitArray128",
    "HostBitArray224",
    "HostBitArray256",
    "HostRing64Tensor",
    "HostRing128Tensor",
    "HostFixed64Tensor",
    "HostFixed128Tensor",
    "HostFloat32Tensor",
    "HostFloat64Tensor",
    "HostInt8Tensor",
    "HostInt16Tensor",
    "HostInt32Tensor",
    "HostInt64Tensor",
    "HostUint8Tensor",
    "HostUint16Tensor",
    "HostUint32Tensor",
    "HostUint64Tensor",
    "HostFixed128AesTensor",
    "HostAesKey",
    "BooleanTensor",
    "Fixed64Tensor",
    "Fixed128Tensor",
    "Float32Tensor",
    "Float64Tensor",
    "Uint64Tensor",
    "ReplicatedRing64Tensor",
    "ReplicatedRing128Tensor",
    "ReplicatedBitTensor",
    "ReplicatedBitArray64",
    "ReplicatedBitArray128",
    "ReplicatedBitArray224",
    "ReplicatedFixed64Tensor",
    "ReplicatedFixed128Tensor",
    "ReplicatedUint64Tensor",
    "ReplicatedAesKey",
    "ReplicatedShape",
    "Mirrored3Ring64Tensor",
    "Mirrored3Ring128Tensor",
    "Mirrored3BitTensor",
    "Mirrored3Fixed64Tensor",
    "Mirrored3Fixed128Tensor",
    "Mirrored3Float32",
    "Mirrored3Float64",
    "AdditiveBitTensor",
    "AdditiveRing64Tensor",
    "AdditiveRing128Tensor",
    "AdditiveShape",
    "Fixed128AesTensor",
    "AesKey",
    "AesTensor",
    "Bit",
    "Float32",
    "Float64",
    "Ring64",
    "Ring128",
    "Fixed",
]
_TYPE_SET = frozenset(TYPE_NAMES)
# deprecated aliases accepted by the parser (computation.rs:363-366)
TYPE_ALIASES = {"Seed": "HostSeed", "PrfKey": "HostPrfKey", "Unit": "HostUnit"}


@dataclass(frozen=True)
class Ty:
    name: str
    inner: Optional[Union[TensorDType, str]] = None

    def __post_init__(self):
        if self.name not in _TYPE_SET:
            raise ValueError(f"unknown type name {self.name!r}")

    def to_textual(self):
        if self.name == "Tensor":
            inner = self.inner if self.inner is not None else UNKNOWN_DTYPE
            return f"Tensor<{inner.to_textual()}>"
        if self.name == "Shape":
            return f"Shape<{self.inner or 'Unknown'}>"
        return self.name

    def __str__(self):
        return self.to_textual()

    @staticmethod
    def from_textual(s: str) -> "Ty":
        s = s.strip()
        if "<" in s:
            name, rest = s.split("<", 1)
            inner = rest.rsplit(">", 1)[0]
            name = name.strip()
            if name == "Tensor":
                return Ty("Tensor", TensorDType.from_textual(inner))
            if name == "Shape":
                inner = inner.strip()
                if inner not in SHAPE_KINDS:
                    raise ValueError(f"unknown shape kind {inner}")
                return Ty("Shape", inner)
            raise ValueError(f"type {name} takes no parameter")
        s = TYPE_ALIASES.get(s, s)
        if s == "Tensor":
            return Ty("Tensor", UNKNOWN_DTYPE)
        return Ty(s)

    # classification helpers used by the interpreter ---------------------------
    @property
    def is_logical_tensor(self):
        return self.name == "Tensor"

    @property
    def dtype(self) -> Optional[TensorDType]:
        return self.inner if self.name == "Tensor" else None


def tensor(dtype: TensorDType) -> Ty:
    return Ty("Tensor", dtype)


UNKNOWN = Ty("Unknown")
HOST_UNIT = Ty("HostUnit")
HOST_SHAPE = Ty("HostShape")
HOST_SEED = Ty("HostSeed")
HOST_PRF_KEY = Ty("HostPrfKey")
HOST_STRING = Ty("HostString")
HOST_RING64 = Ty("HostRing64Tensor")
HOST_RING128 = Ty("HostRing128Tensor")
HOST_BIT = Ty("HostBitTensor")
HOST_FLOAT32 = Ty("HostFloat32Tensor")
HOST_FLOAT64 = Ty("HostFloat64Tensor")


def host_ring(bits: int) -> Ty:
    return HOST_RING64 if bits == 64 else HOST_RING128
