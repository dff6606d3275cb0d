"""Declarative dispatch table for dialect-level operations on replicated and additive
placements.

A row is (operator, placement kind, operand type families) -> kernel; ``lookup`` picks the
first row whose families match the operator's signature.  This is the role of the
reference's ``#[kernel]`` dispatch tables (``moose/src/kernels/*.rs``, e.g. ``arithmetic.rs``
``AddOp``: ``[ReplicatedRing64Tensor, ReplicatedRing64Tensor] -> ...``,
``[HostRing64Tensor, ReplicatedRing64Tensor] -> ...``), so that textual computations below
the logical level -- compiled graphs, hand-written dialect programs -- can use any listed
(op, types) combination on the interpreter.

Families: ``rep_ring`` (ReplicatedRing{64,128}Tensor), ``rep_bit`` (ReplicatedBitTensor),
``rep_bitarray`` (ReplicatedBitArray{64,128,224}: here a boolean sharing of packed words),
``adt_ring`` (AdditiveRing{64,128}Tensor), ``host_ring``/``host_bit`` (public operands),
``host_shape``.  Kernels receive the protocol values (RepTensor / AdtTensor / HV) after the
interpreter moved each operand to the operator's placement, and return one.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from moose_amd.ops import ring as R
from moose_amd.protocols import additive
from moose_amd.protocols import replicated as rep


def family(tyname: str) -> str:
    if tyname.startswith("ReplicatedRing"):
        return "rep_ring"
    if tyname == "ReplicatedBitTensor":
        return "rep_bit"
    if tyname.startswith("ReplicatedBitArray"):
        return "rep_bitarray"
    if tyname.startswith("AdditiveRing"):
        return "adt_ring"
    if tyname.startswith("HostRing"):
        return "host_ring"
    if tyname == "HostBitTensor":
        return "host_bit"
    if tyname == "HostShape":
        return "host_shape"
    return "other"


def ring_bits_of(tyname: str) -> Optional[int]:
    for b in (224, 128, 64):
        if str(b) in tyname:
            return b
    return 1 if "Bit" in tyname else None


@dataclass(frozen=True)
class Kernel:
    op: str
    plc: str  # "rep", "adt" or "host"
    ins: Tuple[str, ...]  # operand families; "*" matches any
    fn: Callable
    variadic: bool = False

    def matches(self, fams: Sequence[str]) -> bool:
        if self.variadic:
            return len(fams) >= 1 and all(self.ins[0] in ("*", f) for f in fams)
        return len(fams) == len(self.ins) and all(p in ("*", f) for p, f in zip(self.ins, fams))


TABLE: List[Kernel] = []
_INDEX: Dict[Tuple[str, str], List[Kernel]] = {}


def kernel(op: str, plc: str, *ins: str, variadic: bool = False):
    def deco(fn):
        k = Kernel(op, plc, tuple(ins), fn, variadic)
        TABLE.append(k)
        _INDEX.setdefault((op, plc), []).append(k)
        return fn
    return deco


def lookup(op: str, plc: str, arg_types: Sequence[str]) -> Optional[Kernel]:
    fams = [family(t) for t in arg_types]
    for k in _INDEX.get((op, plc), ()):
        if k.matches(fams):
            return k
    return None


def ops_for(plc: str) -> List[str]:
    return sorted({k.op for k in TABLE if k.plc == plc})


class Ctx:
    """What a kernel sees: the session, the operator (attributes, signature) and its
    placement."""

    def __init__(self, sess, op):
        self.sess, self.op, self.plc, self.attrs = sess, op, op.placement, op.attrs

    @property
    def ret(self) -> str:
        return self.op.sig.ret.name

    def attr(self, *names, default=None):
        for n in names:
            if n in self.attrs:
                return self.attrs[n]
        return default


def _pub(v):
    return v.v  # a host operand's ring tensor, used as a public value


# --- replicated: arithmetic ---------------------------------------------------------------
for _op, _f in (("Add", rep.add), ("Sub", rep.sub)):
    kernel(_op, "rep", "rep_ring", "rep_ring")(lambda c, x, y, f=_f: f(c.sess, x, y))
    kernel(_op, "rep", "rep_bit", "rep_bit")(lambda c, x, y: rep.xor(c.sess, x, y))
    kernel(_op, "rep", "rep_bitarray", "rep_bitarray")(lambda c, x, y: rep.xor(c.sess, x, y))
kernel("Add", "rep", "rep_ring", "host_ring")(lambda c, x, y: rep.add_public(c.sess, x, _pub(y)))
kernel("Add", "rep", "host_ring", "rep_ring")(lambda c, x, y: rep.add_public(c.sess, y, _pub(x)))
kernel("Sub", "rep", "rep_ring", "host_ring")(lambda c, x, y: rep.sub_public(c.sess, x, _pub(y)))
kernel("Sub", "rep", "host_ring", "rep_ring")(lambda c, x, y: rep.public_sub(c.sess, _pub(x), y))
kernel("Mul", "rep", "rep_ring", "rep_ring")(lambda c, x, y: rep.mul(c.sess, x, y))
kernel("Mul", "rep", "rep_ring", "host_ring")(lambda c, x, y: rep.mul_public(c.sess, x, _pub(y)))
kernel("Mul", "rep", "host_ring", "rep_ring")(lambda c, x, y: rep.mul_public(c.sess, y, _pub(x)))
kernel("Dot", "rep", "rep_ring", "rep_ring")(lambda c, x, y: rep.dot(c.sess, x, y))
kernel("Dot", "rep", "rep_ring", "host_ring")(lambda c, x, y: rep.dot_public(c.sess, x, _pub(y)))
kernel("Dot", "rep", "host_ring", "rep_ring")(
    lambda c, x, y: rep.dot_public(c.sess, y, _pub(x), public_left=True))
kernel("Neg", "rep", "rep_ring")(lambda c, x: rep.neg(c.sess, x))
kernel("Sum", "rep", "rep_ring")(lambda c, x: rep.sum(c.sess, x, c.attr("axis")))
kernel("AddN", "rep", "rep_ring", variadic=True)(lambda c, *xs: _add_n(c, xs))
kernel("Shl", "rep", "rep_ring")(lambda c, x: rep.shl(c.sess, x, int(c.attr("amount"))))
kernel("Shl", "rep", "rep_bitarray")(lambda c, x: rep.shl(c.sess, x, int(c.attr("amount"))))
kernel("TruncPr", "rep", "rep_ring")(
    lambda c, x: rep.trunc_pr(c.sess, x, int(c.attr("amount", "precision", default=0))))
kernel("Abs", "rep", "rep_ring")(lambda c, x: rep.abs_(c.sess, x))
kernel("Relu", "rep", "rep_ring")(lambda c, x: rep.relu(c.sess, x))
for _sel in ("rep_ring", "rep_bit"):  # ring-form or bit-form selector
    kernel("Mux", "rep", _sel, "rep_ring", "rep_ring")(lambda c, s, x, y: rep.mux(c.sess, s, x, y))


def _add_n(c, xs):
    acc = xs[0]
    for x in xs[1:]:
        acc = rep.add(c.sess, acc, x)
    return acc


# --- replicated: boolean ---------------------------------------------------------------
kernel("Xor", "rep", "rep_bit", "rep_bit")(lambda c, x, y: rep.xor(c.sess, x, y))
kernel("Xor", "rep", "rep_bitarray", "rep_bitarray")(lambda c, x, y: rep.xor(c.sess, x, y))
kernel("Xor", "rep", "rep_bit", "host_bit")(lambda c, x, y: rep.add_public(c.sess, x, _pub(y)))
kernel("Xor", "rep", "host_bit", "rep_bit")(lambda c, x, y: rep.add_public(c.sess, y, _pub(x)))
kernel("And", "rep", "rep_bit", "rep_bit")(lambda c, x, y: rep.and_(c.sess, x, y))
kernel("And", "rep", "rep_bitarray", "rep_bitarray")(lambda c, x, y: rep.and_(c.sess, x, y))
kernel("And", "rep", "rep_bit", "host_bit")(lambda c, x, y: rep.mul_public(c.sess, x, _pub(y)))
kernel("And", "rep", "host_bit", "rep_bit")(lambda c, x, y: rep.mul_public(c.sess, y, _pub(x)))
kernel("Or", "rep", "rep_bit", "rep_bit")(
    lambda c, x, y: rep.xor(c.sess, rep.xor(c.sess, x, y), rep.and_(c.sess, x, y)))


# --- replicated: bit decomposition and conversions ---------------------------------------
def _bit_or_ring(c, b):
    """Boolean bit result, or its arithmetic injection when the signature asks for a ring
    (the reference has both kernels for Msb / Equal / EqualZero)."""
    if family(c.ret) == "rep_ring":
        return rep.b2a(c.sess, b, ring_bits_of(c.ret))
    return b


kernel("BitDecompose", "rep", "rep_ring")(lambda c, x: rep.bit_decompose(c.sess, x))
kernel("BitCompose", "rep", "rep_bitarray")(lambda c, x: bit_compose(c.sess, x))
kernel("ShlDim", "rep", "rep_bitarray")(lambda c, x: shl_dim(c.sess, x, int(c.attr("amount")),
                                                             int(c.attr("bit_length", default=x.bits))))
kernel("BitExtract", "rep", "rep_bitarray")(
    lambda c, x: rep.bit_extract(c.sess, x, int(c.attr("bit_idx"))))
kernel("Index", "rep", "rep_bitarray")(lambda c, x: rep.bit_extract(c.sess, x, int(c.attr("index"))))
kernel("RingInject", "rep", "rep_bit")(
    lambda c, x: rep.shl(c.sess, rep.b2a(c.sess, x, ring_bits_of(c.ret)),
                         int(c.attr("bit_idx", default=0))))
kernel("Msb", "rep", "rep_ring")(lambda c, x: _bit_or_ring(c, rep.msb(c.sess, x)))
kernel("EqualZero", "rep", "rep_ring")(lambda c, x: _bit_or_ring(c, rep.equal_zero(c.sess, x)))
kernel("Equal", "rep", "rep_ring", "rep_ring")(
    lambda c, x, y: _bit_or_ring(c, rep.equal(c.sess, x, y)))
kernel("LessThan", "rep", "rep_ring", "rep_ring")(
    lambda c, x, y: _bit_or_ring(c, rep.less(c.sess, x, y)))
kernel("GreaterThan", "rep", "rep_ring", "rep_ring")(
    lambda c, x, y: _bit_or_ring(c, rep.greater(c.sess, x, y)))
kernel("RingCast", "rep", "rep_ring")(lambda c, x: rep.ring_cast(c.sess, x, ring_bits_of(c.ret)))
kernel("AdtToRep", "rep", "adt_ring")(lambda c, y: additive.to_rep(c.sess, c.plc, y))
kernel("Share", "rep", "host_ring")(lambda c, x: rep.share(c.sess, c.plc, x, kind="arith"))
kernel("Share", "rep", "host_bit")(lambda c, x: rep.share(c.sess, c.plc, x, kind="bool"))

# shape / linear ops are share-wise
for _op in ("Reshape", "ExpandDims", "Squeeze", "Transpose", "Slice", "IndexAxis", "Broadcast",
            "Concat"):
    kernel(_op, "rep", "rep_ring", variadic=_op == "Concat")(
        lambda c, *xs, p=_op: _local(c, p, xs))
    kernel(_op, "rep", "rep_bit", variadic=_op == "Concat")(
        lambda c, *xs, p=_op: _local(c, p, xs))


def _local(c, prim, xs):
    from moose_amd.runtime.graph_executor import prim_attrs

    attrs = prim_attrs(c.op, dict(c.attrs), c.sess.device)
    attrs.pop("bits", None)
    attrs.pop("device", None)
    if len(xs) == 1:
        return rep.local(c.sess, xs[0], prim, **attrs)
    x0 = xs[0]  # Concat: share-wise over the party vectors
    s0 = c.sess.p(prim, x0.plc, *[x.s0 for x in xs], **attrs)
    s1 = c.sess.p(prim, x0.plc, *[x.s1 for x in xs], **attrs)
    return rep.RepTensor(x0.plc, x0.bits, x0.kind, s0, s1)


def bit_compose(sess, x):
    """Packed boolean sharing of k bits -> arithmetic sharing of the k-bit value: the bit
    planes (one kernel) go through ONE batched b2a (one multiplication round for all k
    bits) and are summed with weights 2^i (one kernel) -- reference ``bits.rs``
    ``BitComposeOp`` (per-bit RingInject + sum)."""
    k = x.bits
    planes = rep.RepTensor(x.plc, 1, "bool", sess.p("BitSplit", x.plc, x.s0, start=0, count=k),
                           sess.p("BitSplit", x.plc, x.s1, start=0, count=k))
    a = rep.b2a(sess, planes, k)
    w = [1 << i for i in range(k)]
    return rep.RepTensor(x.plc, k, "arith", sess.p("WeightedSum", x.plc, a.s0, weights=w, bits=k),
                         sess.p("WeightedSum", x.plc, a.s1, weights=w, bits=k))


def shl_dim(sess, x, amount: int, bit_length: int):
    """Shift a bit array along its bit dimension (reference ``ShlDimOp``): bit i moves to
    i + amount, the low ``amount`` bits become zero -- a word shift of the packed form,
    masked to ``bit_length`` bits."""
    y = rep.shl(sess, x, amount)
    if bit_length < x.bits:
        mask = R.fill((), (1 << bit_length) - 1, x.bits, sess.device)
        y = rep.mul_public(sess, y, mask)
    return y


# --- additive --------------------------------------------------------------------------------
kernel("RepToAdt", "adt", "rep_ring")(lambda c, x: additive.from_rep(c.sess, x, c.plc))
kernel("Add", "adt", "adt_ring", "adt_ring")(lambda c, x, y: additive.add(c.sess, x, y))
kernel("Sub", "adt", "adt_ring", "adt_ring")(lambda c, x, y: additive.sub(c.sess, x, y))
kernel("Add", "adt", "adt_ring", "host_ring")(
    lambda c, x, y: additive.add_public(c.sess, x, _pub(y)))
kernel("Add", "adt", "host_ring", "adt_ring")(
    lambda c, x, y: additive.add_public(c.sess, y, _pub(x)))
kernel("Mul", "adt", "adt_ring", "host_ring")(
    lambda c, x, y: additive.mul_public(c.sess, x, _pub(y)))
kernel("Mul", "adt", "host_ring", "adt_ring")(
    lambda c, x, y: additive.mul_public(c.sess, y, _pub(x)))
kernel("Neg", "adt", "adt_ring")(lambda c, x: additive.neg(c.sess, x))
kernel("Shl", "adt", "adt_ring")(lambda c, x: additive.shl(c.sess, x, int(c.attr("amount"))))
kernel("Share", "adt", "host_ring")(lambda c, x: additive.share(c.sess, c.plc, x))

# --- host: opening ---------------------------------------------------------------------------
for _f in ("rep_ring", "rep_bit", "rep_bitarray"):
    kernel("Reveal", "host", _f)(lambda c, x: rep.reveal(c.sess, x, c.plc.owner))
kernel("Reveal", "host", "adt_ring")(lambda c, x: additive.reveal(c.sess, x, c.plc.owner))
