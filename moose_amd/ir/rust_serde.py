"""Rust-layout binary computations: the reference's own ``to_bincode`` / ``to_msgpack`` bytes.

Parity: reference ``NamedComputation::{to,from}_bincode`` and ``{to,from}_msgpack`` /
``{to,from}_disk`` (``moose/src/computation.rs:1797-1874``), i.e. serde-derived
serialisation of ``NamedComputation { operations: Vec<Operation> }`` with
``Operation { name, kind: Operator, inputs, placement }`` (``:1656-1666``).  This is the
format the reference's ``elk compile -f bincode|msgpack`` writes and ``comet``/``rudolph``
and the filesystem choreography read (``bin/elk/main.rs:211-245``,
``choreography/filesystem.rs:219-227``); ``moose_amd/ir/bincode.py`` / ``serde.py`` are
this framework's own (more compact) binary forms.

The data model is walked once per type declaration of the reference:

* ``Operator`` -- newtype variants in ``operators![..]`` order (:828-914) over ``XOp``
  structs ``{sig, attributes...}`` with the attribute types of their declarations
  (``usize`` / ``u32`` / ``u64`` / ``Option<_>`` / ``Vec<usize>`` / ``String`` /
  ``[u8; 16]`` keys / ``SliceInfo`` / ``Constant``);
* ``Signature`` (:620-650), ``Ty`` (:334-345: ``Unknown``, the ``values![..]`` list,
  then the scalar pseudo-types; ``Shape(TensorShape)`` and ``Tensor(TensorDType)`` carry
  an inner enum, ``logical/mod.rs:17-43``), ``Placement`` (:1626) with ``Role(String)``;
* ``Constant`` (``constants![..]`` then ``Bit, Float32, Float64, Ring64, Ring128,
  Fixed``): host tensors are ``HostTensor<T>(ArcArrayD<T>, HostPlacement)`` with
  ndarray's serde form ``{v: u8 = 1, dim: [usize], data: [T]}``; ``HostBitTensor`` is a
  ``BitArrayRepr { data: BitVec<u8, Lsb0>, dim }`` with bitvec's serde form
  ``{order, head: {width, index}, bits, data}``.

Two encoders of that one walk:

* ``bincode`` (bincode 1.3 default options): little-endian fixed-width integers
  (``usize`` as u64), u64 length prefixes, u32 variant indices, u8 option tags, fixed
  arrays and structs without prefixes;
* ``msgpack`` (rmp-serde 1.1 ``to_vec``): structs as arrays, enum variants by name
  (unit variant = the name string, newtype/struct variant = a one-entry map), ``None`` =
  nil, ``u128`` as 16-byte big-endian bin, integers in their most compact form.

Parity is unpinned: the reference ships no binary fixtures, so the layout follows the
type declarations and the serde rules above (``tests/test_rust_serde.py`` pins hand-built
byte strings of those rules).  Values this IR has and the Rust enums lack (our fused
``EXTENSION_OPERATORS``, Broadcast/Reshape's optional ``shape``) raise / are dropped.
Constants: text-parsed constants in the reference carry the placement ``"TODO"``
(``textual/parsing.rs:631``), which the encoder writes too; ``Fixed`` carries one
precision in Rust (``FixedpointConstant {value, precision}``), the fractional one here.
"""
from __future__ import annotations

import struct
from typing import List

import numpy as np

from moose_amd.ir.computation import Computation
from moose_amd.ir.computation import Constant
from moose_amd.ir.computation import HostPlacement
from moose_amd.ir.computation import Operation
from moose_amd.ir.computation import Signature
from moose_amd.ir.computation import placement_from
from moose_amd.ir.operators import OPERATORS
from moose_amd.ir.types import SHAPE_KINDS
from moose_amd.ir.types import TYPE_NAMES
from moose_amd.ir.types import TensorDType
from moose_amd.ir.types import Ty


class RustSerdeError(ValueError):
    pass


# enum variant lists, in declaration order --------------------------------------------
OPERATOR_VARIANTS = list(OPERATORS)  # same order as operators![..]
TY_VARIANTS = list(TYPE_NAMES)       # Unknown, values![..], Bit .. Fixed
SIG_VARIANTS = ["Nullary", "Unary", "Binary", "Ternary", "Variadic"]
PLACEMENT_VARIANTS = ["Host", "Replicated", "Additive", "Mirrored3"]
DTYPE_VARIANTS = ["Fixed64", "Fixed128", "Float32", "Float64", "Bool", "Uint64", "Unknown"]
CONSTANT_VARIANTS = ["RawShape", "RawSeed", "RawPrfKey", "String", "HostBitTensor",
                     "HostRing64Tensor", "HostRing128Tensor", "HostFloat32Tensor",
                     "HostFloat64Tensor", "HostInt8Tensor", "HostInt16Tensor",
                     "HostInt32Tensor", "HostInt64Tensor", "HostUint8Tensor",
                     "HostUint16Tensor", "HostUint32Tensor", "HostUint64Tensor",
                     "Bit", "Float32", "Float64", "Ring64", "Ring128", "Fixed"]
_CONST_OF_KIND = {"HostShape": "RawShape", "HostSeed": "RawSeed", "HostPrfKey": "RawPrfKey",
                  "HostString": "String"}
_KIND_OF_CONST = {v: k for k, v in _CONST_OF_KIND.items()}

# Rust attribute types of each operator's fields after ``sig`` (computation.rs:922-1547);
# attributes of this IR not in the Rust struct are dropped (Broadcast/Reshape ``shape``)
ATTR_TYPES = {
    "AtLeast2D": [("to_column_vector", "bool")],
    "BitExtract": [("bit_idx", "usize")],
    "Concat": [("axis", "u32")],
    "Constant": [("value", "const")],
    "DeriveSeed": [("sync_key", "key")],
    "ExpandDims": [("axis", "vec_usize")],
    "IndexAxis": [("axis", "usize"), ("index", "usize")],
    "Input": [("arg_name", "string")],
    "Mean": [("axis", "opt_u32")],
    "Output": [("tag", "string")],
    "Receive": [("rendezvous_key", "key"), ("sender", "string")],
    "RingFixedpointArgmax": [("axis", "usize"), ("upmost_index", "usize")],
    "RingFixedpointDecode": [("scaling_base", "u64"), ("scaling_exp", "u32")],
    "RingFixedpointEncode": [("scaling_base", "u64"), ("scaling_exp", "u32")],
    "RingInject": [("bit_idx", "usize")],
    "RingFixedpointMean": [("axis", "opt_u32"), ("scaling_base", "u64"), ("scaling_exp", "u32")],
    "Sample": [("max_value", "opt_u64")],
    "SampleSeeded": [("max_value", "opt_u64")],
    "Select": [("axis", "usize")],
    "Send": [("rendezvous_key", "key"), ("receiver", "string")],
    "Shl": [("amount", "usize")],
    "Shr": [("amount", "usize")],
    "Slice": [("slice", "slice")],
    "Squeeze": [("axis", "opt_usize")],
    "Sum": [("axis", "opt_usize")],
    "FixedpointEncode": [("fractional_precision", "u32"), ("integral_precision", "u32")],
    "FixedpointDecode": [("fractional_precision", "u32")],
    "Argmax": [("axis", "usize"), ("upmost_index", "usize")],
    "Fill": [("value", "const")],
    "Index": [("index", "usize")],
    "Softmax": [("axis", "usize"), ("upmost_index", "usize")],
    "ShlDim": [("amount", "usize"), ("bit_length", "usize")],
    "TruncPr": [("amount", "u32")],
}

# host tensor constants: element codec (bincode struct code, msgpack kind)
_ELEM = {
    "HostRing64Tensor": ("<Q", "uint", np.uint64), "HostRing128Tensor": (None, "u128", object),
    "HostFloat32Tensor": ("<f", "f32", np.float32), "HostFloat64Tensor": ("<d", "f64", np.float64),
    "HostInt8Tensor": ("<b", "int", np.int8), "HostInt16Tensor": ("<h", "int", np.int16),
    "HostInt32Tensor": ("<i", "int", np.int32), "HostInt64Tensor": ("<q", "int", np.int64),
    "HostUint8Tensor": ("<B", "uint", np.uint8), "HostUint16Tensor": ("<H", "uint", np.uint16),
    "HostUint32Tensor": ("<I", "uint", np.uint32), "HostUint64Tensor": ("<Q", "uint", np.uint64),
}
_ARRAY_FORMAT_VERSION = 1  # ndarray's serde ARRAY_FORMAT_VERSION
_BITVEC_ORDER = "bitvec::order::Lsb0"
_CONST_PLACEMENT = "TODO"
M128 = (1 << 128) - 1


# ---------------------------------------------------------------------------------------
# format writers / readers: the serde data model primitives
# ---------------------------------------------------------------------------------------
class _BincodeW:
    def __init__(self):
        self.out = []

    def _p(self, fmt, v):
        self.out.append(struct.pack(fmt, v))

    def boolean(self, v):
        self._p("<B", 1 if v else 0)

    def uint(self, v, bits):
        self._p({8: "<B", 16: "<H", 32: "<I", 64: "<Q"}[bits], v)

    def sint(self, v, bits):
        self._p({8: "<b", 16: "<h", 32: "<i", 64: "<q"}[bits], v)

    def u128(self, v):
        self.out.append(int(v & M128).to_bytes(16, "little"))

    def f32(self, v):
        self._p("<f", v)

    def f64(self, v):
        self._p("<d", v)

    def string(self, s):
        b = s.encode()
        self._p("<Q", len(b))
        self.out.append(b)

    def seq(self, n):
        self._p("<Q", n)

    def tuple(self, n):  # fixed arrays, tuple structs
        pass

    def struct(self, n):
        pass

    def none(self):
        self._p("<B", 0)

    def some(self):
        self._p("<B", 1)

    def unit_variant(self, idx, name):
        self._p("<I", idx)

    def variant(self, idx, name):  # newtype / struct variant header
        self._p("<I", idx)

    def bytes_fixed(self, b):  # [u8; N]
        self.out.append(bytes(b))

    def raw_elems(self, arr, code):  # a homogeneous run of fixed-width scalars
        self.out.append(np.ascontiguousarray(arr, dtype=np.dtype(code)).tobytes())

    def getvalue(self):
        return b"".join(self.out)


class _MsgpackW:
    def __init__(self):
        self.out = bytearray()

    def _uint(self, v):
        o = self.out
        if v < 0x80:
            o.append(v)
        elif v <= 0xFF:
            o += b"\xcc" + struct.pack(">B", v)
        elif v <= 0xFFFF:
            o += b"\xcd" + struct.pack(">H", v)
        elif v <= 0xFFFFFFFF:
            o += b"\xce" + struct.pack(">I", v)
        else:
            o += b"\xcf" + struct.pack(">Q", v)

    def _sint(self, v):
        if v >= 0:
            return self._uint(v)
        o = self.out
        if v >= -32:
            o += struct.pack(">b", v)
        elif v >= -128:
            o += b"\xd0" + struct.pack(">b", v)
        elif v >= -32768:
            o += b"\xd1" + struct.pack(">h", v)
        elif v >= -(1 << 31):
            o += b"\xd2" + struct.pack(">i", v)
        else:
            o += b"\xd3" + struct.pack(">q", v)

    def _len(self, n, fix, base16):
        if n < 16:
            self.out.append(fix | n)
        elif n <= 0xFFFF:
            self.out += bytes([base16]) + struct.pack(">H", n)
        else:
            self.out += bytes([base16 + 1]) + struct.pack(">I", n)

    def boolean(self, v):
        self.out.append(0xC3 if v else 0xC2)

    def uint(self, v, bits):
        self._uint(int(v))

    def sint(self, v, bits):
        self._sint(int(v))

    def u128(self, v):
        self.out += b"\xc4\x10" + int(v & M128).to_bytes(16, "big")

    def f32(self, v):
        self.out += b"\xca" + struct.pack(">f", v)

    def f64(self, v):
        self.out += b"\xcb" + struct.pack(">d", v)

    def string(self, s):
        b = s.encode()
        n = len(b)
        if n < 32:
            self.out.append(0xA0 | n)
        elif n <= 0xFF:
            self.out += b"\xd9" + struct.pack(">B", n)
        elif n <= 0xFFFF:
            self.out += b"\xda" + struct.pack(">H", n)
        else:
            self.out += b"\xdb" + struct.pack(">I", n)
        self.out += b

    def seq(self, n):
        self._len(n, 0x90, 0xDC)

    tuple = seq
    struct = seq

    def none(self):
        self.out.append(0xC0)

    def some(self):
        pass

    def unit_variant(self, idx, name):
        self.string(name)

    def variant(self, idx, name):
        self._len(1, 0x80, 0xDE)
        self.string(name)

    def bytes_fixed(self, b):
        self.seq(len(b))
        for x in bytes(b):
            self._uint(x)

    def raw_elems(self, arr, code):
        f = self.f32 if code == "<f" else self.f64 if code == "<d" else None
        for x in np.asarray(arr).reshape(-1).tolist():
            if f is not None:
                f(x)
            else:
                self._sint(int(x))

    def getvalue(self):
        return bytes(self.out)


class _BincodeR:
    def __init__(self, data: bytes):
        self.b = memoryview(data)
        self.i = 0

    def _take(self, n):
        if self.i + n > len(self.b):
            raise RustSerdeError("truncated bincode input")
        v = self.b[self.i:self.i + n]
        self.i += n
        return v

    def _u(self, fmt, n):
        return struct.unpack(fmt, self._take(n))[0]

    def boolean(self):
        v = self._u("<B", 1)
        if v > 1:
            raise RustSerdeError(f"invalid bool byte {v}")
        return bool(v)

    def uint(self, bits):
        return self._u({8: "<B", 16: "<H", 32: "<I", 64: "<Q"}[bits], bits // 8)

    def sint(self, bits):
        return self._u({8: "<b", 16: "<h", 32: "<i", 64: "<q"}[bits], bits // 8)

    def u128(self):
        return int.from_bytes(self._take(16), "little")

    def f32(self):
        return self._u("<f", 4)

    def f64(self):
        return self._u("<d", 8)

    def string(self):
        n = self._u("<Q", 8)
        try:
            return bytes(self._take(n)).decode()
        except UnicodeDecodeError as e:
            raise RustSerdeError(f"invalid utf-8 string: {e}") from e

    def seq(self):
        return self._u("<Q", 8)

    def tuple(self, n):
        pass

    def struct(self, n):
        pass

    def option(self):
        t = self._u("<B", 1)
        if t > 1:
            raise RustSerdeError(f"invalid option tag {t}")
        return t == 1

    def variant(self, names, units=()):
        idx = self._u("<I", 4)
        if idx >= len(names):
            raise RustSerdeError(f"variant index {idx} out of range for {names[0]}..")
        return idx

    def bytes_fixed(self, n):
        return bytes(self._take(n))

    def raw_elems(self, n, code):
        w = struct.calcsize(code)
        return np.frombuffer(bytes(self._take(n * w)), dtype=np.dtype(code)).copy()

    def done(self):
        return self.i == len(self.b)


class _MsgpackR:
    def __init__(self, data: bytes):
        self.b = bytes(data)
        self.i = 0

    def _byte(self):
        if self.i >= len(self.b):
            raise RustSerdeError("truncated msgpack input")
        v = self.b[self.i]
        self.i += 1
        return v

    def _take(self, n):
        if self.i + n > len(self.b):
            raise RustSerdeError("truncated msgpack input")
        v = self.b[self.i:self.i + n]
        self.i += n
        return v

    def _peek(self):
        if self.i >= len(self.b):
            raise RustSerdeError("truncated msgpack input")
        return self.b[self.i]

    def _int(self):
        t = self._byte()
        if t < 0x80:
            return t
        if t >= 0xE0:
            return t - 0x100
        fmt = {0xCC: ">B", 0xCD: ">H", 0xCE: ">I", 0xCF: ">Q",
               0xD0: ">b", 0xD1: ">h", 0xD2: ">i", 0xD3: ">q"}.get(t)
        if fmt is None:
            raise RustSerdeError(f"expected an integer, found msgpack tag 0x{t:02x}")
        return struct.unpack(fmt, self._take(struct.calcsize(fmt)))[0]

    def _len(self, fix_lo, fix_hi, t16, what):
        t = self._byte()
        if fix_lo <= t <= fix_hi:
            return t - fix_lo
        if t == t16:
            return struct.unpack(">H", self._take(2))[0]
        if t == t16 + 1:
            return struct.unpack(">I", self._take(4))[0]
        raise RustSerdeError(f"expected a {what}, found msgpack tag 0x{t:02x}")

    def boolean(self):
        t = self._byte()
        if t not in (0xC2, 0xC3):
            raise RustSerdeError(f"expected a bool, found msgpack tag 0x{t:02x}")
        return t == 0xC3

    def uint(self, bits):
        v = self._int()
        if v < 0 or v >> bits:
            raise RustSerdeError(f"integer {v} out of range for u{bits}")
        return v

    def sint(self, bits):
        v = self._int()
        if not -(1 << (bits - 1)) <= v < (1 << (bits - 1)):
            raise RustSerdeError(f"integer {v} out of range for i{bits}")
        return v

    def u128(self):
        t = self._byte()
        if t != 0xC4 or self._byte() != 16:
            raise RustSerdeError("expected a 16-byte bin (u128)")
        return int.from_bytes(self._take(16), "big")

    def _float(self):
        t = self._byte()
        if t == 0xCA:
            return struct.unpack(">f", self._take(4))[0]
        if t == 0xCB:
            return struct.unpack(">d", self._take(8))[0]
        raise RustSerdeError(f"expected a float, found msgpack tag 0x{t:02x}")

    f32 = _float
    f64 = _float

    def string(self):
        t = self._byte()
        if 0xA0 <= t <= 0xBF:
            n = t - 0xA0
        elif t in (0xD9, 0xDA, 0xDB):
            w = {0xD9: 1, 0xDA: 2, 0xDB: 4}[t]
            n = int.from_bytes(self._take(w), "big")
        else:
            raise RustSerdeError(f"expected a string, found msgpack tag 0x{t:02x}")
        try:
            return self._take(n).decode()
        except UnicodeDecodeError as e:
            raise RustSerdeError(f"invalid utf-8 string: {e}") from e

    def seq(self):
        return self._len(0x90, 0x9F, 0xDC, "array")

    def tuple(self, n):
        got = self.seq()
        if got != n:
            raise RustSerdeError(f"expected an array of {n}, found {got}")

    struct = tuple

    def option(self):
        if self._peek() == 0xC0:
            self.i += 1
            return False
        return True

    def variant(self, names, units=()):
        t = self._peek()
        if 0xA0 <= t <= 0xBF or t in (0xD9, 0xDA, 0xDB):  # unit variant by name
            name = self.string()
            if name not in units:
                raise RustSerdeError(f"{name!r} is not a unit variant here")
        else:
            n = self._len(0x80, 0x8F, 0xDE, "map (enum variant)")
            if n != 1:
                raise RustSerdeError(f"an enum variant is a one-entry map, found {n} entries")
            name = self.string()
        try:
            return names.index(name)
        except ValueError:
            raise RustSerdeError(f"unknown variant {name!r} of {names[0]}..") from None

    def bytes_fixed(self, n):
        self.tuple(n)
        return bytes(self.uint(8) for _ in range(n))

    def raw_elems(self, n, code):
        if code in ("<f", "<d"):
            vals = [self._float() for _ in range(n)]
        else:
            vals = [self._int() for _ in range(n)]
        return np.asarray(vals, dtype=np.dtype(code))

    def done(self):
        return self.i == len(self.b)


# ---------------------------------------------------------------------------------------
# encoders (one walk for both formats)
# ---------------------------------------------------------------------------------------
def _w_ty(w, t: Ty):
    idx = TY_VARIANTS.index(t.name)
    if t.name == "Shape":
        w.variant(idx, "Shape")
        inner = t.inner or "Unknown"
        w.unit_variant(SHAPE_KINDS.index(inner), inner)
    elif t.name == "Tensor":
        w.variant(idx, "Tensor")
        d = t.inner if t.inner is not None else TensorDType("Unknown")
        di = DTYPE_VARIANTS.index(d.kind)
        if d.is_fixed:
            w.variant(di, d.kind)
            w.struct(2)
            w.uint(d.integral_precision, 32)
            w.uint(d.fractional_precision, 32)
        else:
            w.unit_variant(di, d.kind)
    else:
        w.unit_variant(idx, t.name)


def _sig_variant(sig: Signature):
    if sig.variadic:
        return 4
    if len(sig.args) > 3:
        raise RustSerdeError(f"no Rust signature takes {len(sig.args)} arguments")
    return len(sig.args)


def _w_sig(w, sig: Signature):
    v = _sig_variant(sig)
    w.variant(v, SIG_VARIANTS[v])
    tys = list(sig.args) + [sig.ret]
    w.struct(len(tys))
    for t in tys:
        _w_ty(w, t)


def _w_host_placement(w, owner):
    w.struct(1)
    w.string(owner)


def _w_placement(w, plc):
    kind = type(plc).__name__.replace("Placement", "")
    idx = PLACEMENT_VARIANTS.index(kind)
    w.variant(idx, kind)
    if isinstance(plc, HostPlacement):
        _w_host_placement(w, plc.owner)
    else:
        w.struct(1)
        w.tuple(len(plc.owners))
        for o in plc.owners:
            w.string(o)


def _w_ndarray(w, a: np.ndarray, elem):
    code, mk, _ = elem
    w.struct(3)
    w.uint(_ARRAY_FORMAT_VERSION, 8)
    w.seq(a.ndim)
    for d in a.shape:
        w.uint(int(d), 64)
    w.seq(a.size)
    if mk == "u128":
        for x in a.reshape(-1).tolist():
            w.u128(int(x))
    else:
        w.raw_elems(a.reshape(-1), code)


def _w_constant(w, c: Constant):
    k = c.kind
    rk = _CONST_OF_KIND.get(k, k)
    if rk not in CONSTANT_VARIANTS:
        raise RustSerdeError(f"constant kind {k} has no Rust Constant variant")
    w.variant(CONSTANT_VARIANTS.index(rk), rk)
    v = c.value
    if rk == "RawShape":
        w.seq(len(v))
        for d in v:
            w.uint(int(d), 64)
    elif rk in ("RawSeed", "RawPrfKey"):
        b = bytes(v)
        if len(b) != 16:
            raise RustSerdeError(f"{k} is 16 bytes, found {len(b)}")
        w.tuple(16)
        w.bytes_fixed(b)
    elif rk == "String":
        w.string(v)
    elif rk == "HostBitTensor":
        a = np.asarray(v, dtype=np.uint8)
        w.tuple(2)
        w.struct(2)  # BitArrayRepr { data: BitVec<u8, Lsb0>, dim: IxDyn }
        bits = a.reshape(-1) & 1
        w.struct(4)  # bitvec "BitSeq" { order, head, bits, data }
        w.string(_BITVEC_ORDER)
        w.struct(2)  # BitIdx { width, index }
        w.uint(8, 8)
        w.uint(0, 8)
        w.uint(int(bits.size), 64)
        packed = np.packbits(bits, bitorder="little") if bits.size else np.zeros(0, np.uint8)
        w.seq(packed.size)
        w.raw_elems(packed, "<B")
        w.seq(a.ndim)
        for d in a.shape:
            w.uint(int(d), 64)
        _w_host_placement(w, _CONST_PLACEMENT)
    elif rk in _ELEM:
        elem = _ELEM[rk]
        a = np.asarray(v, dtype=elem[2])
        w.tuple(2)
        _w_ndarray(w, a, elem)
        _w_host_placement(w, _CONST_PLACEMENT)
    elif rk == "Bit":
        w.uint(int(v), 8)
    elif rk == "Float32":
        w.f32(float(v))
    elif rk == "Float64":
        w.f64(float(v))
    elif rk == "Ring64":
        w.uint(int(v) & ((1 << 64) - 1), 64)
    elif rk == "Ring128":
        w.u128(int(v))
    elif rk == "Fixed":
        val, _i, frac = v
        w.struct(2)
        w.f64(float(val))
        w.uint(int(frac), 64)


def _w_slice_elem(w, s):
    start, end, step = s
    w.struct(3)
    w.sint(int(start), 64)
    for o in (end, step):
        if o is None:
            w.none()
        else:
            w.some()
            w.sint(int(o), 64)


def _w_attr(w, kind, v, op):
    if kind == "bool":
        w.boolean(bool(v))
    elif kind in ("usize", "u64"):
        w.uint(int(v), 64)
    elif kind == "u32":
        w.uint(int(v), 32)
    elif kind.startswith("opt_"):
        if v is None:
            w.none()
        else:
            w.some()
            w.uint(int(v), 32 if kind == "opt_u32" else 64)
    elif kind == "vec_usize":
        v = list(v) if isinstance(v, (list, tuple)) else [v]
        w.seq(len(v))
        for x in v:
            w.uint(int(x), 64)
    elif kind == "string":
        w.string(v)
    elif kind == "key":
        b = bytes(v)
        if len(b) != 16:
            raise RustSerdeError(f"{op.name}: keys are 16 bytes")
        w.tuple(16)
        w.bytes_fixed(b)
    elif kind == "slice":
        elems = v if isinstance(v, list) else [v]
        w.seq(len(elems))
        for s in elems:
            _w_slice_elem(w, s)
    elif kind == "const":
        _w_constant(w, v)
    else:  # pragma: no cover - table error
        raise RustSerdeError(f"unknown attribute kind {kind}")


def _w_operation(w, op: Operation):
    if op.kind not in OPERATORS:
        raise RustSerdeError(
            f"operation {op.name}: {op.kind} is this framework's fused kernel, not a Rust "
            "Operator variant (serialise the computation before lowering)")
    w.struct(4)
    w.string(op.name)
    attrs = ATTR_TYPES.get(op.kind, [])
    w.variant(OPERATOR_VARIANTS.index(op.kind), op.kind)
    w.struct(1 + len(attrs))
    _w_sig(w, op.sig)
    for an, ak in attrs:
        if an not in op.attrs:
            raise RustSerdeError(f"operation {op.name}: attribute {an} missing")
        _w_attr(w, ak, op.attrs[an], op)
    w.seq(len(op.inputs))
    for i in op.inputs:
        w.string(i)
    _w_placement(w, op.placement)


def _encode(comp: Computation, w) -> bytes:
    w.struct(1)  # NamedComputation { operations }
    w.seq(len(comp.operations))
    for op in comp.operations:
        _w_operation(w, op)
    return w.getvalue()


# ---------------------------------------------------------------------------------------
# decoders
# ---------------------------------------------------------------------------------------
def _r_ty(r) -> Ty:
    idx = r.variant(TY_VARIANTS, units=tuple(n for n in TY_VARIANTS if n not in ("Shape", "Tensor")))
    name = TY_VARIANTS[idx]
    if name == "Shape":
        k = r.variant(list(SHAPE_KINDS), units=SHAPE_KINDS)
        return Ty("Shape", SHAPE_KINDS[k])
    if name == "Tensor":
        di = r.variant(DTYPE_VARIANTS, units=DTYPE_VARIANTS[2:])
        kind = DTYPE_VARIANTS[di]
        if kind in ("Fixed64", "Fixed128"):
            r.struct(2)
            return Ty("Tensor", TensorDType(kind, r.uint(32), r.uint(32)))
        return Ty("Tensor", TensorDType(kind))
    return Ty(name)


def _r_sig(r) -> Signature:
    v = r.variant(SIG_VARIANTS)
    n = {0: 1, 1: 2, 2: 3, 3: 4, 4: 2}[v]
    r.struct(n)
    tys = [_r_ty(r) for _ in range(n)]
    return Signature(tuple(tys[:-1]), tys[-1], variadic=v == 4)


def _r_host_placement(r) -> str:
    r.struct(1)
    return r.string()


def _r_placement(r):
    idx = r.variant(PLACEMENT_VARIANTS)
    kind = PLACEMENT_VARIANTS[idx]
    if kind == "Host":
        return HostPlacement(_r_host_placement(r))
    n = 2 if kind == "Additive" else 3
    r.struct(1)
    r.tuple(n)
    return placement_from(kind, [r.string() for _ in range(n)])


def _r_dims(r) -> List[int]:
    return [r.uint(64) for _ in range(r.seq())]


def _r_ndarray(r, elem) -> np.ndarray:
    code, mk, npt = elem
    r.struct(3)
    ver = r.uint(8)
    if ver != _ARRAY_FORMAT_VERSION:
        raise RustSerdeError(f"unknown ndarray format version {ver}")
    dims = _r_dims(r)
    n = r.seq()
    if n != int(np.prod(dims, dtype=np.int64)):
        raise RustSerdeError(f"ndarray of shape {dims} with {n} elements")
    if mk == "u128":
        a = np.empty(n, dtype=object)
        for i in range(n):
            a[i] = r.u128()
    else:
        a = r.raw_elems(n, code).astype(npt)
    return a.reshape(dims)


def _r_constant(r) -> Constant:
    idx = r.variant(CONSTANT_VARIANTS)
    rk = CONSTANT_VARIANTS[idx]
    kind = _KIND_OF_CONST.get(rk, rk)
    if rk == "RawShape":
        return Constant(kind, _r_dims(r))
    if rk in ("RawSeed", "RawPrfKey"):
        r.tuple(16)
        return Constant(kind, r.bytes_fixed(16))
    if rk == "String":
        return Constant(kind, r.string())
    if rk == "HostBitTensor":
        r.tuple(2)
        r.struct(2)
        r.struct(4)
        order = r.string()
        if order != _BITVEC_ORDER:
            raise RustSerdeError(f"bit order {order!r} (expected {_BITVEC_ORDER})")
        r.struct(2)
        width, head = r.uint(8), r.uint(8)
        if width != 8 or head != 0:
            raise RustSerdeError(f"bit vector head ({width}, {head}) is not byte-aligned")
        nbits = r.uint(64)
        packed = r.raw_elems(r.seq(), "<B").astype(np.uint8)
        dims = _r_dims(r)
        _r_host_placement(r)
        bits = np.unpackbits(packed, bitorder="little")[:nbits]
        if bits.size != int(np.prod(dims, dtype=np.int64)):
            raise RustSerdeError(f"bit tensor of shape {dims} with {bits.size} bits")
        return Constant(kind, bits.astype(np.uint8).reshape(dims))
    if rk in _ELEM:
        r.tuple(2)
        a = _r_ndarray(r, _ELEM[rk])
        _r_host_placement(r)
        return Constant(kind, a)
    if rk == "Bit":
        return Constant(kind, r.uint(8))
    if rk == "Float32":
        return Constant(kind, r.f32())
    if rk == "Float64":
        return Constant(kind, r.f64())
    if rk == "Ring64":
        return Constant(kind, r.uint(64))
    if rk == "Ring128":
        return Constant(kind, r.u128())
    r.struct(2)  # Fixed
    val = r.f64()
    return Constant(kind, (val, 0, r.uint(64)))


def _r_attr(r, kind):
    if kind == "bool":
        return r.boolean()
    if kind in ("usize", "u64"):
        return r.uint(64)
    if kind == "u32":
        return r.uint(32)
    if kind.startswith("opt_"):
        return r.uint(32 if kind == "opt_u32" else 64) if r.option() else None
    if kind == "vec_usize":
        return [r.uint(64) for _ in range(r.seq())]
    if kind == "string":
        return r.string()
    if kind == "key":
        r.tuple(16)
        return r.bytes_fixed(16)
    if kind == "slice":
        out = []
        for _ in range(r.seq()):
            r.struct(3)
            start = r.sint(64)
            end = r.sint(64) if r.option() else None
            step = r.sint(64) if r.option() else None
            out.append((start, end, step))
        return out[0] if len(out) == 1 else out
    if kind == "const":
        return _r_constant(r)
    raise RustSerdeError(f"unknown attribute kind {kind}")  # pragma: no cover


def _r_operation(r) -> Operation:
    r.struct(4)
    name = r.string()
    kind = OPERATOR_VARIANTS[r.variant(OPERATOR_VARIANTS)]
    attrs_t = ATTR_TYPES.get(kind, [])
    r.struct(1 + len(attrs_t))
    sig = _r_sig(r)
    attrs = {an: _r_attr(r, ak) for an, ak in attrs_t}
    for an, ak in OPERATORS[kind]:  # IR-only optional attributes (Broadcast/Reshape shape)
        if an not in attrs and ak.startswith("opt_"):
            attrs[an] = None
    inputs = [r.string() for _ in range(r.seq())]
    plc = _r_placement(r)
    return Operation(name, kind, inputs, plc, sig, attrs)


def _decode(r) -> Computation:
    r.struct(1)
    ops = [_r_operation(r) for _ in range(r.seq())]
    if not r.done():
        raise RustSerdeError("trailing bytes after the computation")
    return Computation(ops)


# ---------------------------------------------------------------------------------------
# public API
# ---------------------------------------------------------------------------------------
def to_rust_bincode(comp: Computation) -> bytes:
    """``NamedComputation::to_bincode`` bytes of ``comp``."""
    return _encode(comp, _BincodeW())


def from_rust_bincode(data: bytes) -> Computation:
    """Inverse of :func:`to_rust_bincode` (``NamedComputation::from_bincode``)."""
    return _decode(_BincodeR(data))


def to_rust_msgpack(comp: Computation) -> bytes:
    """``NamedComputation::to_msgpack`` / ``to_disk`` bytes of ``comp`` (rmp-serde)."""
    return _encode(comp, _MsgpackW())


def from_rust_msgpack(data: bytes) -> Computation:
    """Inverse of :func:`to_rust_msgpack` (``from_msgpack`` / ``from_disk``)."""
    return _decode(_MsgpackR(data))
