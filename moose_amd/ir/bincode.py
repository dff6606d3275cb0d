"""Bincode-style binary serialisation of computations.

Parity: reference ``Computation::{to,from}_bincode`` (``moose/src/computation.rs:1837-1844``),
used by ``elk compile -f bincode`` (``bin/elk/main.rs:216,245``) and the filesystem
choreography (``choreography/filesystem.rs:227``).  The encoding follows bincode's rules
-- little-endian fixed-width integers, ``u64`` length prefixes for strings/sequences,
``u32`` enum variant tags, ``u8`` option tags, struct fields in declaration order
without names -- applied to this framework's IR: operators and placements are enum
variants (tag = index in the operator catalogue / placement list), attributes follow
the operator's schema order.  The reference's exact Rust type layout is not
reproduced (parity unpinned: the reference ships no bincode fixtures to pin it).
"""
from __future__ import annotations

import struct

import numpy as np

from moose_amd.ir.computation import Computation
from moose_amd.ir.computation import Constant
from moose_amd.ir.computation import Operation
from moose_amd.ir.computation import Signature
from moose_amd.ir.computation import TENSOR_CONSTANT_NP
from moose_amd.ir.computation import placement_from
from moose_amd.ir.operators import ALL_OPERATORS
from moose_amd.ir.types import Ty

MAGIC = b"MXBC\x01\x00\x00\x00"
_OPS = list(ALL_OPERATORS)
_OP_INDEX = {k: i for i, k in enumerate(_OPS)}
_PLACEMENTS = ["Host", "Replicated", "Additive", "Mirrored3"]
_CONSTS = list(TENSOR_CONSTANT_NP) + ["HostShape", "HostString", "HostSeed", "HostPrfKey",
                                      "Ring64", "Ring128", "Bit", "Float32", "Float64", "Fixed"]
_CONST_INDEX = {k: i for i, k in enumerate(_CONSTS)}
_NP_ELEM = {"HostRing128Tensor": 16}
M64 = (1 << 64) - 1


class BincodeError(ValueError):
    pass


class _W:
    def __init__(self):
        self.parts = []

    def u8(self, v):
        self.parts.append(struct.pack("<B", v))

    def u32(self, v):
        self.parts.append(struct.pack("<I", v))

    def u64(self, v):
        self.parts.append(struct.pack("<Q", v))

    def i64(self, v):
        self.parts.append(struct.pack("<q", v))

    def f32(self, v):
        self.parts.append(struct.pack("<f", v))

    def f64(self, v):
        self.parts.append(struct.pack("<d", v))

    def u128(self, v):
        v &= (1 << 128) - 1
        self.parts.append(struct.pack("<QQ", v & M64, v >> 64))

    def raw(self, b):
        self.parts.append(bytes(b))

    def bytes_(self, b):
        self.u64(len(b))
        self.raw(b)

    def str_(self, s):
        self.bytes_(s.encode())

    def opt(self, v, f):
        if v is None:
            self.u8(0)
        else:
            self.u8(1)
            f(v)


class _R:
    def __init__(self, data):
        self.b = memoryview(data)
        self.i = 0

    def take(self, n):
        if self.i + n > len(self.b):
            raise BincodeError("truncated bincode payload")
        out = self.b[self.i:self.i + n]
        self.i += n
        return out

    def _s(self, fmt, n):
        return struct.unpack(fmt, self.take(n))[0]

    def u8(self):
        return self._s("<B", 1)

    def u32(self):
        return self._s("<I", 4)

    def u64(self):
        return self._s("<Q", 8)

    def i64(self):
        return self._s("<q", 8)

    def f32(self):
        return self._s("<f", 4)

    def f64(self):
        return self._s("<d", 8)

    def u128(self):
        lo, hi = struct.unpack("<QQ", self.take(16))
        return lo | (hi << 64)

    def bytes_(self):
        return bytes(self.take(self.u64()))

    def str_(self):
        return self.bytes_().decode()

    def opt(self, f):
        tag = self.u8()
        if tag > 1:
            raise BincodeError(f"bad option tag {tag}")
        return f() if tag else None


# -- constants ---------------------------------------------------------------------
def _w_const(w: _W, c: Constant):
    w.u32(_CONST_INDEX[c.kind])
    k, v = c.kind, c.value
    if k in TENSOR_CONSTANT_NP:
        a = np.asarray(v)
        w.u64(a.ndim)
        for d in a.shape:
            w.u64(d)
        if k == "HostRing128Tensor":
            for e in a.reshape(-1):
                w.u128(int(e))
        else:
            w.raw(np.ascontiguousarray(a, dtype=np.dtype(TENSOR_CONSTANT_NP[k]).newbyteorder("<"))
                  .tobytes())
    elif k == "HostShape":
        w.u64(len(v))
        for d in v:
            w.u64(int(d))
    elif k == "HostString":
        w.str_(v)
    elif k in ("HostSeed", "HostPrfKey"):
        w.bytes_(bytes(v))
    elif k == "Ring64":
        w.u64(int(v) & M64)
    elif k == "Ring128":
        w.u128(int(v))
    elif k == "Bit":
        w.u8(int(v) & 1)
    elif k == "Float32":
        w.f32(float(v))
    elif k == "Float64":
        w.f64(float(v))
    elif k == "Fixed":
        val, i, f = v
        w.f64(float(val))
        w.u32(int(i))
        w.u32(int(f))
    else:  # pragma: no cover - catalogue and encoder are kept in sync
        raise BincodeError(f"cannot encode constant {k}")


def _r_const(r: _R) -> Constant:
    idx = r.u32()
    if idx >= len(_CONSTS):
        raise BincodeError(f"bad constant tag {idx}")
    k = _CONSTS[idx]
    if k in TENSOR_CONSTANT_NP:
        shape = tuple(r.u64() for _ in range(r.u64()))
        n = int(np.prod(shape)) if shape else 1
        if k == "HostRing128Tensor":
            arr = np.array([r.u128() for _ in range(n)], dtype=object).reshape(shape)
        else:
            dt = np.dtype(TENSOR_CONSTANT_NP[k]).newbyteorder("<")
            arr = np.frombuffer(r.take(n * dt.itemsize), dtype=dt).astype(
                TENSOR_CONSTANT_NP[k]).reshape(shape)
        return Constant(k, arr)
    if k == "HostShape":
        return Constant(k, tuple(r.u64() for _ in range(r.u64())))
    if k == "HostString":
        return Constant(k, r.str_())
    if k in ("HostSeed", "HostPrfKey"):
        return Constant(k, r.bytes_())
    if k == "Ring64":
        return Constant(k, r.u64())
    if k == "Ring128":
        return Constant(k, r.u128())
    if k == "Bit":
        return Constant(k, r.u8())
    if k == "Float32":
        return Constant(k, r.f32())
    if k == "Float64":
        return Constant(k, r.f64())
    val = r.f64()
    return Constant("Fixed", (val, r.u32(), r.u32()))


# -- attributes ---------------------------------------------------------------------
def _w_slice(w: _W, s):
    w.i64(int(s[0]))
    w.opt(s[1], lambda x: w.i64(int(x)))
    w.opt(s[2], lambda x: w.i64(int(x)))


def _w_attr(w: _W, kind: str, v):
    if kind == "int":
        w.i64(int(v))
    elif kind == "opt_int":
        w.opt(v, lambda x: w.i64(int(x)))
    elif kind in ("ints", "opt_ints"):
        def seq(xs):
            w.u64(len(xs))
            for x in xs:
                w.i64(int(x))
        if kind == "opt_ints":
            w.opt(v, seq)
        else:
            seq(v)
    elif kind == "bool":
        w.u8(1 if v else 0)
    elif kind == "str":
        w.str_(v)
    elif kind == "key":
        b = bytes(v)
        if len(b) != 16:
            raise BincodeError("rendezvous/sync keys are 16 bytes")
        w.raw(b)
    elif kind == "const":
        _w_const(w, v)
    elif kind == "slice":
        if isinstance(v, list):
            w.u32(1)
            w.u64(len(v))
            for s in v:
                _w_slice(w, s)
        else:
            w.u32(0)
            _w_slice(w, v)
    else:  # pragma: no cover
        raise BincodeError(f"unknown attribute kind {kind}")


def _r_slice(r: _R):
    return (r.i64(), r.opt(r.i64), r.opt(r.i64))


def _r_attr(r: _R, kind: str):
    if kind == "int":
        return r.i64()
    if kind == "opt_int":
        return r.opt(r.i64)
    if kind in ("ints", "opt_ints"):
        def seq():
            return [r.i64() for _ in range(r.u64())]
        return r.opt(seq) if kind == "opt_ints" else seq()
    if kind == "bool":
        return bool(r.u8())
    if kind == "str":
        return r.str_()
    if kind == "key":
        return bytes(r.take(16))
    if kind == "const":
        return _r_const(r)
    if kind == "slice":
        if r.u32() == 1:
            return [_r_slice(r) for _ in range(r.u64())]
        return _r_slice(r)
    raise BincodeError(f"unknown attribute kind {kind}")


# -- computation ----------------------------------------------------------------------
def to_bincode(comp: Computation) -> bytes:
    w = _W()
    w.raw(MAGIC)
    w.u64(len(comp.operations))
    for op in comp.operations:
        w.str_(op.name)
        w.u32(_OP_INDEX[op.kind])
        w.u64(len(op.inputs))
        for i in op.inputs:
            w.str_(i)
        plc = op.placement
        w.u32(_PLACEMENTS.index(type(plc).__name__.replace("Placement", "")))
        for o in plc.owners:
            w.str_(o)
        w.u8(1 if op.sig.variadic else 0)
        w.u64(len(op.sig.args))
        for t in op.sig.args:
            w.str_(t.to_textual())
        w.str_(op.sig.ret.to_textual())
        for an, ak in ALL_OPERATORS[op.kind]:
            _w_attr(w, ak, op.attrs.get(an))
    return b"".join(w.parts)


def from_bincode(data: bytes) -> Computation:
    r = _R(data)
    if bytes(r.take(len(MAGIC))) != MAGIC:
        raise BincodeError("not a moosex bincode computation")
    ops = []
    tys = {}

    def ty(s):
        t = tys.get(s)
        if t is None:
            t = tys[s] = Ty.from_textual(s)
        return t

    for _ in range(r.u64()):
        name = r.str_()
        k = r.u32()
        if k >= len(_OPS):
            raise BincodeError(f"bad operator tag {k}")
        kind = _OPS[k]
        inputs = [r.str_() for _ in range(r.u64())]
        p = r.u32()
        if p >= len(_PLACEMENTS):
            raise BincodeError(f"bad placement tag {p}")
        pk = _PLACEMENTS[p]
        owners = [r.str_() for _ in range({"Host": 1, "Additive": 2}.get(pk, 3))]
        variadic = bool(r.u8())
        args = tuple(ty(r.str_()) for _ in range(r.u64()))
        ret = ty(r.str_())
        attrs = {an: _r_attr(r, ak) for an, ak in ALL_OPERATORS[kind]}
        ops.append(Operation(name, kind, inputs, placement_from(pk, owners),
                             Signature(args, ret, variadic), attrs))
    if r.i != len(r.b):
        raise BincodeError("trailing bytes after the computation")
    return Computation(ops)
