"""Replicated fixed-point arithmetic and the non-linear functions built on it.

Parity: reference ``moose/src/fixedpoint/ops.rs`` (precision bookkeeping, TruncPr after
mul/dot) and ``moose/src/replicated/{division,exp,log,sqrt,softmax,argmax}.rs``.

A :class:`RepFixed` is an arithmetic RSS tensor whose ring elements encode
``value * 2^frac``.  Non-linear functions share one normalisation primitive:

* :func:`_top_bit_onehot` -- bit-decompose |x| (packed words), prefix-OR from the top
  (log2 k boolean ANDs), one-hot of the leading bit, then ONE batched B2A of the relevant
  bit planes.  From the arithmetic one-hot bits t_j any public function of the exponent
  (2^-j, 2^(j/2), j ...) is a local weighted sum.
* mantissa m in [0.5, 1) = x * 2^(f-1-j)  ->  polynomial (Estrin/power-tree, log depth)
  for 1/m, sqrt(m), log2(m).

This replaces the reference's Goldschmidt reciprocal (division.rs:5-86) and int2fl log
(log.rs:9-106) with fewer sequential rounds.  exp uses 2^x = 2^int * 2^frac with the
integer part from B2A'd exponent bits (product tree, log depth -- the reference folds
sequentially, exp.rs:155) and a polynomial for the fraction; negative inputs use the
2^-int factors directly instead of a reciprocal.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from functools import lru_cache

import numpy as np
import torch

from moose_amd.ops import ring as R
from moose_amd.protocols import replicated as rep
from moose_amd.protocols.replicated import RepTensor
from moose_amd.runtime.session import PV
from moose_amd.runtime.values import MV


@dataclass
class RepFixed:
    t: RepTensor
    frac: int
    integ: int

    @property
    def bits(self):
        return self.t.bits

    @property
    def plc(self):
        return self.t.plc


def _pub(v):
    """Public operand payload: MV -> its value."""
    return v.v if isinstance(v, MV) else v


def _encode_const(sess, value: float, frac: int, bits: int):
    return R.fill((), int(round(value * (1 << frac))), bits, sess.device)


def _with(x: RepFixed, t: RepTensor) -> RepFixed:
    return RepFixed(t, x.frac, x.integ)


# ---------------------------------------------------------------------------
# linear ops
# ---------------------------------------------------------------------------
def local(sess, x, prim, *extra, **attrs):
    if isinstance(x, RepFixed):
        return _with(x, local(sess, x.t, prim, *extra, **attrs))
    if extra:
        # extra positional (e.g. Select mask) are public values
        pub = [sess.public(x.plc, e) for e in extra]
        return RepTensor(x.plc, x.bits, x.kind, sess.p(prim, x.plc, x.s0, *pub, **attrs),
                         sess.p(prim, x.plc, x.s1, *pub, **attrs))
    return rep.local(sess, x, prim, **attrs)


def add(sess, x, y, px=None, py=None):
    if px is not None:
        return _with(y, rep.add_public(sess, y.t, px))
    if py is not None:
        return _with(x, rep.add_public(sess, x.t, py))
    return _with(x, rep.add(sess, x.t, y.t))


def sub(sess, x, y, px=None, py=None):
    if px is not None:
        return _with(y, rep.add_public(sess, rep.neg(sess, y.t), px))
    if py is not None:
        return _with(x, rep.sub_public(sess, x.t, py))
    return _with(x, rep.sub(sess, x.t, y.t))


def neg(sess, x: RepFixed) -> RepFixed:
    return _with(x, rep.neg(sess, x.t))


def mul(sess, x, y, px=None, py=None, f=None):
    if px is not None:
        x, y, px, py = y, MV(None, px), None, px
    if py is not None:
        z = rep.mul_public(sess, x.t, _pub(py))
    else:
        return _with(x, rep.mul_trunc(sess, x.t, y.t, f if f is not None else x.frac))
    return _with(x, rep.trunc_pr(sess, z, f if f is not None else x.frac))


def dot(sess, x, y, px=None, py=None, f=None):
    m = f if f is not None else (y.frac if px is not None else x.frac)
    if (px is not None or py is not None) and 0 < m <= 63 and _jobs_ok(
            sess, (y if px is not None else x).t):
        return _dot_public_trunc_jobs(sess, x, y, px, py, m)
    if px is not None:
        z = rep.dot_public(sess, y.t, px, public_left=True)
        base = y
    elif py is not None:
        z = rep.dot_public(sess, x.t, py)
        base = x
    else:
        return _with(x, rep.dot_trunc(sess, x.t, y.t, f if f is not None else x.frac))
    return _with(base, rep.trunc_pr(sess, z, f if f is not None else base.frac))


def _dot_public_trunc_jobs(sess, x, y, px, py, m):
    """A secret x public fixed-point product on a per-party session: the GEMM of this
    party's FIRST share component only (an additive sharing of the product) and its TruncPr
    through the batched tail -- one GEMM and 3 kernels (the generic path multiplies both
    components, then runs TruncPr on the replicated product)."""
    base = y if px is not None else x
    t = base.t
    plc, bits = t.plc, t.bits
    pc = sess.public(plc, _pub(px if px is not None else py))
    v0 = sess.p("Dot", plc, pc, t.s0) if px is not None else sess.p("Dot", plc, t.s0, pc)
    if DEFER_DOT_TRUNC:
        # the tail waits for the reader: the shares complete with the same tail when read,
        # the sigmoid's decomposition and a reveal take the untruncated value instead
        return _with(base, rep.PendingTrunc(sess, plc, bits, v0.v, m))
    nonces = _tail_nonces(sess, plc)
    r = rep.tail_job(sess, plc, bits, m, nonces, v0,
                     lambda o0, o1: R.MulJob(1, o0, o1, a=v0.v.data.contiguous()))
    return _with(base, r)


def dot_many(sess, pairs, f=None):
    """Several independent secret x secret fixed-point products of equal shapes at once:
    the operands are stacked on a new leading axis, so the k products share one batched
    MFMA GEMM launch (batch = parties x k), one zero-share/reshare round and one TruncPr
    -- instead of k of each (the interpreter batches independent Dot ops this way)."""
    if len(pairs) == 1:
        return [dot(sess, pairs[0][0], pairs[0][1], f=f)]
    x0 = pairs[0][0]
    X = _stack_operands(sess, [x for x, _ in pairs])
    Y = _stack_operands(sess, [y for _, y in pairs])
    m = f if f is not None else x0.frac
    if getattr(sess, "party_dot_trunc", None) is not None and not getattr(
            sess, "is_simulated", True):
        # one party per process / thread: the batched GEMM, then ONE dot tail (zero share
        # + reshare folded into TruncPr: 2 rounds) for all k products
        T = _with(x0, rep.dot_trunc(sess, X.t, Y.t, m, nbatch=1))
    else:
        Z = rep.dot(sess, X.t, Y.t, nbatch=1)
        T = _with(x0, rep.trunc_pr(sess, Z, m))
    return [local(sess, T, "IndexAxis", axis=0, index=i) for i in range(len(pairs))]


def _stack_operands(sess, xs):
    """Stack on a new leading axis; k uses of ONE operand become a zero-copy broadcast view
    where the session supports it (the GEMM reads it with batch stride 0) -- k products are
    still computed, only the k physical copies of the operand are avoided."""
    rep0 = getattr(sess, "p_repeat0", None)
    if rep0 is not None and all(x is xs[0] for x in xs):
        t = xs[0].t if isinstance(xs[0], RepFixed) else xs[0]
        r = RepTensor(t.plc, t.bits, t.kind, rep0(t.s0, len(xs)), rep0(t.s1, len(xs)))
        return _with(xs[0], r) if isinstance(xs[0], RepFixed) else r
    return concat(sess, [local(sess, x, "ExpandDims", axis=[0]) for x in xs], 0)


def mul_const(sess, x: RepFixed, c: float) -> RepFixed:
    """x * c for a public real constant (one truncation)."""
    cv = int(round(c * (1 << x.frac)))
    return _with(x, rep.mul_public_trunc(sess, x.t, _encode_const(sess, c, x.frac, x.bits),
                                         x.frac, value=cv))


def add_const(sess, x: RepFixed, c: float) -> RepFixed:
    return _with(x, rep.add_public(sess, x.t, _encode_const(sess, c, x.frac, x.bits)))


def const_sub(sess, c: float, x: RepFixed) -> RepFixed:
    """c - x for a public real constant (one share-wise kernel)."""
    return _with(x, rep.lincomb(sess, [(-1, x.t)], const=_encode_const(sess, c, x.frac, x.bits)))


def ring_binary(sess, kind, x, y, px=None, py=None):
    if kind == "Add":
        if px is not None:
            return rep.add_public(sess, y, px)
        if py is not None:
            return rep.add_public(sess, x, py)
        return rep.add(sess, x, y)
    if kind == "Sub":
        if py is not None:
            return rep.sub_public(sess, x, py)
        if px is not None:
            return rep.add_public(sess, rep.neg(sess, y), px)
        return rep.sub(sess, x, y)
    if kind == "Mul":
        if py is not None:
            return rep.mul_public(sess, x, py)
        if px is not None:
            return rep.mul_public(sess, y, px)
        return rep.mul(sess, x, y)
    if kind == "Dot":
        if py is not None:
            return rep.dot_public(sess, x, py)
        if px is not None:
            return rep.dot_public(sess, y, px, public_left=True)
        return rep.dot(sess, x, y)
    raise NotImplementedError(kind)


def cast(sess, x: RepFixed, target) -> RepFixed:
    bits = target.ring_bits
    t = x.t
    df = target.fractional_precision - x.frac
    if df < 0:
        t = rep.trunc_pr(sess, t, -df)
    if bits != t.bits:
        if bits < t.bits:
            t = rep.ring_cast(sess, t, bits)
        else:
            raise NotImplementedError("replicated ring extension 64 -> 128")
    if df > 0:
        t = rep.shl(sess, t, df)
    return RepFixed(t, target.fractional_precision, target.integral_precision)


def mean(sess, x: RepFixed, axis):
    s = local(sess, x, "Sum", axis=axis)
    shape = shape_of(sess, x)
    n = math.prod(shape) if axis is None else shape[axis]
    return mul_const(sess, s, 1.0 / n)


def concat(sess, xs, axis):
    ts = [x.t if isinstance(x, RepFixed) else x for x in xs]
    plc = ts[0].plc
    s0 = sess.p("Concat", plc, *[t.s0 for t in ts], axis=axis)
    s1 = sess.p("Concat", plc, *[t.s1 for t in ts], axis=axis)
    t = RepTensor(plc, ts[0].bits, ts[0].kind, s0, s1)
    return _with(xs[0], t) if isinstance(xs[0], RepFixed) else t


def broadcast_to(sess, x, shape):
    """Share-wise broadcast of a (fixed-point) sharing to ``shape`` (no-op if equal)."""
    if tuple(shape_of(sess, x)) == tuple(shape):
        return x
    return local(sess, x, "Broadcast", shape=tuple(shape))


def shape_of(sess, x):
    t = x.t if isinstance(x, RepFixed) else x
    if isinstance(t, MV):
        return tuple(t.v.shape)
    if isinstance(t, rep.PendingTrunc) and not t.completed:  # without completing it
        return sess.p_shape(PV(t.plc, t.v_add))
    return sess.p_shape(t.s0)


def static_shape(sess, x):
    """shape_of, or None where the shape is only known at run time (shape-polymorphic
    lowering without arg_specs)."""
    try:
        return shape_of(sess, x)
    except ValueError:
        return None


def broadcast_like(sess, small: RepTensor, big: RepTensor) -> RepTensor:
    """``small`` broadcast to ``big``'s shape: a static Broadcast when the shape is known,
    else BroadcastLike, which reads the shape from ``big`` when the lowered graph runs."""
    shape = static_shape(sess, big)
    if shape is not None:
        return rep.local(sess, small, "Broadcast", shape=tuple(shape))
    s0, s1 = rep._sharewise(sess, "BroadcastLike", small.plc, (small.s0, small.s1),
                            (big.s0, big.s1))
    return RepTensor(small.plc, small.bits, small.kind, s0, s1)


# ---------------------------------------------------------------------------
# comparisons and selection
# ---------------------------------------------------------------------------
def _as_rep(sess, x, like: RepFixed):
    if isinstance(x, RepFixed):
        return x
    return RepFixed(rep.from_public(sess, like.plc, _pub(x), like.bits), like.frac, like.integ)


def compare(sess, kind, x, y, px=None, py=None) -> RepTensor:
    """[x < y] / [x > y] as a boolean bit sharing."""
    if px is not None:
        diff = rep.add_public(sess, rep.neg(sess, _t(y)), px)  # px - y
    elif py is not None:
        diff = rep.sub_public(sess, _t(x), py)  # x - py
    else:
        diff = rep.sub(sess, _t(x), _t(y))
    if kind == "Less":
        return rep.msb(sess, diff)
    # x > y  <=>  y - x < 0
    return rep.msb(sess, rep.neg(sess, diff))


def _t(x):
    return x.t if isinstance(x, RepFixed) else x


def mux(sess, s, x, y):
    """s ? x : y  (s boolean bit or arithmetic 0/1)."""
    if isinstance(x, RepFixed):
        return _with(x, rep.mux(sess, s, x.t, y.t))
    return rep.mux(sess, s, x, y)


# opt-in (MOOSEX_SIGN_WIDTH=1): take the sign of a fixed(i, f) value from bit i + f of its
# ring element, running the sign's adder over those low bits only.  That is only right while
# |x| < 2^i, and i is a NOMINAL bound (mul and dot keep it while the value grows), so by
# default relu / abs / sign_bit use the ring's msb as the reference does
# (replicated/exp.rs, fixedpoint ops: rep.msb over all bits).
SIGN_WIDTH = os.environ.get("MOOSEX_SIGN_WIDTH", "0") == "1"


# exp's adder carries only over the bits its planes read (MOOSEX_EXP_WIDTH=0: all bits)
EXP_WIDTH = os.environ.get("MOOSEX_EXP_WIDTH", "1") != "0"


def _value_width(x: RepFixed):
    w = x.integ + x.frac + 1
    return w if SIGN_WIDTH and 2 < w < x.bits else None


def sign_bit(sess, x: RepFixed) -> RepTensor:
    """Arithmetic 0/1 sharing of [x < 0]."""
    return rep.less_than_zero_arith(sess, x.t, width=_value_width(x))


def relu(sess, x: RepFixed) -> RepFixed:
    s = sign_bit(sess, x)
    return _with(x, rep.sub(sess, x.t, rep.mul(sess, s, x.t)))


def abs_(sess, x: RepFixed) -> RepFixed:
    s = sign_bit(sess, x)
    return _with(x, rep.negate_where(sess, s, x.t))


def _stack0(sess, xs):
    """Equal-shape values stacked on a new leading axis (one concat per share)."""
    return concat(sess, [local(sess, x, "ExpandDims", axis=[0]) for x in xs], 0)


def _unstack0(sess, x, n):
    return [local(sess, x, "IndexAxis", axis=0, index=i) for i in range(n)]


def maximum(sess, xs):
    """Elementwise maximum of a list: a tree of (less, mux) whose every level is ONE
    stacked comparison and ONE stacked mux over all its pairs (log2(n) protocol
    instances in all, not n - 1)."""
    xs = list(xs)
    while len(xs) > 1:
        h = len(xs) // 2
        if h == 1:
            a, b = xs[0], xs[1]
            nxt = [mux(sess, rep.msb(sess, rep.sub(sess, a.t, b.t)), b, a)]  # a < b
        else:
            A, B = _stack0(sess, xs[0:2 * h:2]), _stack0(sess, xs[1:2 * h:2])
            lt = rep.msb(sess, rep.sub(sess, A.t, B.t))
            nxt = _unstack0(sess, mux(sess, lt, B, A), h)
        if len(xs) % 2:
            nxt.append(xs[-1])
        xs = nxt
    return xs[0]


# ---------------------------------------------------------------------------
# normalisation: leading-bit one-hot
# ---------------------------------------------------------------------------
def _or(sess, a: RepTensor, b: RepTensor) -> RepTensor:
    return rep.xor(sess, rep.xor(sess, a, b), rep.and_(sess, a, b))


def _top_bit_onehot(sess, x: RepTensor, lo: int, hi: int) -> RepTensor:
    """For x >= 0 (arithmetic): arithmetic 0/1 sharings t_j, j in [lo, hi), stacked on a
    new leading axis, with t_j = 1 iff bit j is the leading one of x."""
    bits = x.bits
    bd = rep.bit_decompose(sess, x)
    p = bd
    d = 1
    while d < bits:
        p = _or(sess, p, rep.local(sess, p, "Shr", amount=d))
        d *= 2
    onehot = rep.xor(sess, p, rep.local(sess, p, "Shr", amount=1))
    return rep.b2a_planes(sess, onehot, lo, hi - lo, bits)


def _weighted(sess, t: RepTensor, weights, bits) -> RepTensor:
    """sum_j w_j t_j over the leading axis (public integer weights, mod 2^bits)."""
    w = [int(v) % (1 << bits) for v in weights]
    s0, s1 = rep._sharewise(sess, "WeightedSum", t.plc, (t.s0, t.s1), weights=w, bits=bits)
    return RepTensor(t.plc, bits, "arith", s0, s1)


def _normalize(sess, x: RepFixed):
    """x > 0 -> (m, t, lo) with m = x * 2^(f-1-j) in [0.5, 1) (fixed, frac f) and t the
    arithmetic one-hot of the leading bit position j in [lo, lo + len)."""
    f, bits = x.frac, x.bits
    hi = min(bits - 1, f + x.integ + 1)
    lo = 0
    t = _top_bit_onehot(sess, x.t, lo, hi)
    # scale factor 2^(f-1-j) as fixed point: weight 2^(2f-1-j) (needs j <= 2f-1)
    weights = [(1 << (2 * f - 1 - j)) if 2 * f - 1 - j >= 0 else 0 for j in range(lo, hi)]
    F = RepFixed(_weighted(sess, t, weights, bits), f, x.integ)
    m = mul(sess, x, F)
    return m, t, lo, hi


# ---------------------------------------------------------------------------
# polynomials (log-depth power tree, public coefficients)
# ---------------------------------------------------------------------------
def poly_eval(sess, x: RepFixed, coeffs, shift: int = 0) -> RepFixed:
    """sum_k c_k x^k (divided by 2^shift: the final TruncPr drops ``shift`` more bits, so
    a halving of the result costs no extra round).  The powers stay stacked on a leading
    axis P = [x, x^2, ...]: level by level x^(h+1..h+m) = x^h * P[0:m] is ONE stacked
    multiplication (depth ceil(log2 n) rounds), and the sum is one public weighted sum over
    P + one TruncPr."""
    n = len(coeffs) - 1
    f, bits = x.frac, x.bits
    if n > 1 and _rows_ok(sess, x):
        return _poly_eval_rows(sess, x, coeffs, shift)
    if n > 1 and 0 < f + shift <= 63 and _jobs_ok(sess, x.t):
        return _poly_eval_jobs(sess, x, coeffs, shift)
    P = local(sess, x, "ExpandDims", axis=[0])
    have = 1
    while have < n:
        m = min(2 * have, n) - have
        xh = local(sess, P, "Slice", slice=(have - 1, have, None))
        # m copies of x^h on the stacking axis (a concat, so no static shape is needed)
        left = xh if m == 1 else concat(sess, [xh] * m, 0)
        right = P if m == have else local(sess, P, "Slice", slice=(0, m, None))
        P = concat(sess, [P, mul(sess, left, right)], 0)
        have += m
    acc = _weighted(sess, P.t, [int(round(c * (1 << f))) for c in coeffs[1:]], bits)
    if _party_tail(sess) and 0 < f + shift <= 63 and x.t.kind == "arith":
        # per-party sessions: TruncPr of the weighted sum's additive shares (each party's
        # first share component) with the dot's tail -- as _merged_exp_tail does, and
        # bitwise what the batched form (_poly_eval_jobs) computes
        ex = local(sess, RepFixed(acc, f, x.integ), "ExpandDims", axis=[0]).t
        acc = local(sess, _tail_trunc(sess, x.t.plc, ex.s0, bits, f + shift), "IndexAxis",
                    axis=0, index=0)
    else:
        acc = rep.trunc_pr(sess, acc, f + shift)
    return add_const(sess, RepFixed(acc, f, x.integ), coeffs[0] / (1 << shift))


def _party_tail(sess) -> bool:
    """One party per process / thread (SPMD, in-process parties) with the dot's folded tail."""
    return (not getattr(sess, "is_simulated", True) and getattr(sess, "party_dot_trunc", None)
            is not None and os.environ.get("MOOSEX_DOT_TAIL", "1") != "0")


def _poly_eval_jobs(sess, x: RepFixed, coeffs, shift: int = 0) -> RepFixed:
    """poly_eval for one party on the batched tail (csrc/rss_jobs.hip): each power level is
    the tail's three kernels reading and writing a preallocated power stack, and the
    weighted sum's TruncPr one more (the weighted sum of the stack rows one kernel) --
    bitwise the generic per-party levels (mul_trunc of the stacked operands) and final
    TruncPr of the weighted sum's additive shares."""
    from moose_amd.parallel.spmd import Remote

    n = len(coeffs) - 1
    f, bits, t = x.frac, x.bits, x.t
    plc = t.plc
    weights = [int(round(c * (1 << f))) for c in coeffs[1:]]
    member = sess.party_index(plc) is not None
    L = max(1, math.prod(sess.p_shape(t.s0))) if member else 1
    st = _Stack(t.s0.v.data, t.s1.v.data, n - 1, bits) if member else None
    have = 1
    while have < n:
        m = min(2 * have, n) - have
        nonces = _tail_nonces(sess, plc)
        if member:  # each level's round-2 sums ride in the next level's round 0
            sess.party_jobs(plc, _power_jobs(st, have, m, L), L, bits, f, nonces, defer=True)
        have += m
    nonces = _tail_nonces(sess, plc)
    if member:
        sess.party_jobs_flush(plc)  # the acc job's weighted sum reads the rows directly
        acc0, acc1 = torch.empty_like(st.x0), torch.empty_like(st.x0)
        sess.party_jobs(plc, [_acc_job(st, weights, n, L, acc0, acc1)], L, bits, f + shift,
                        nonces)
        acc = RepTensor(plc, bits, "arith", PV(plc, R.RT(acc0, bits)), PV(plc, R.RT(acc1, bits)))
    else:
        r = PV(plc, Remote(bits))
        acc = RepTensor(plc, bits, "arith", r, r)
    return add_const(sess, RepFixed(acc, f, x.integ), coeffs[0] / (1 << shift))


def _poly_powers_sum(sess, x: RepFixed, coeffs, finish=None):
    """sum_{k>=1} w_k x^k (w_k = c_k at x's fractional bits) WITHOUT truncation: the power
    levels of _poly_eval_jobs, then the weighted sum of the replicated powers -- both share
    components, so the result is replicated (scale 2^2f) and costs no round."""
    n = len(coeffs) - 1
    f, bits, t = x.frac, x.bits, x.t
    plc = t.plc
    weights = [int(round(c * (1 << f))) for c in coeffs[1:]]
    member = sess.party_index(plc) is not None
    L = max(1, math.prod(sess.p_shape(t.s0))) if member else 1
    st = _Stack(t.s0.v.data, t.s1.v.data, n - 1, bits) if member else None
    have = 1
    while have < n:
        m = min(2 * have, n) - have
        nonces = _tail_nonces(sess, plc)
        if member:  # each level's round-2 sums ride in the next level's round 0
            sess.party_jobs(plc, _power_jobs(st, have, m, L), L, bits, f, nonces, defer=True)
        have += m
    if member:
        sess.party_jobs_flush(plc)  # the last level's sums, before the rows are read
        rows = RepTensor(plc, bits, "arith", PV(plc, R.RT(st.s0, bits)), PV(plc, R.RT(st.s1, bits)))
    else:
        from moose_amd.parallel.spmd import Remote

        r = PV(plc, Remote(bits))
        rows = RepTensor(plc, bits, "arith", r, r)
    if finish is not None:  # (c0, m2, c2): W + c0 and m2 (W + c0) + c2 in one launch
        c0, m2, c2 = finish
        got = _wsum(sess, rows, weights[1:], x=t, wx=weights[0], cblk=(c0,),
                    second=(m2, (m2 * c0 + c2)))
        if got is not None:
            return got
        big = rep.add_public(sess, rep.lincomb(sess, [(weights[0], t),
                                                      (1, _weighted(sess, rows, weights[1:],
                                                                    bits))]),
                             R.fill((), c0, bits, sess.device))
        return big, rep.lincomb(sess, [(m2, big)], const=R.fill((), c2, bits, sess.device))
    acc = _weighted(sess, rows, weights[1:], bits)
    return rep.lincomb(sess, [(weights[0], t), (1, acc)])


def _wsum(sess, rows, weights, x=None, wx=0, cblk=(0,), second=None, nrows=None,
          lead=False):
    """Per-party fused local step (csrc/wsum_pair.h): s = sum_k weights[k] rows[k] + wx x
    over both share components in ONE launch; returns the RepTensor s + cblk[b] (blocks on
    a new leading axis when len(cblk) > 1, the public constants on this party's copies of
    x_0) and, with ``second`` = (m2, c2), also m2 s + c2 -- with ``lead``, as block 0 of
    ONE RepTensor of 1 + len(cblk) blocks.  Bitwise the composition of the separate
    weighted sum / multiply / add / lincomb steps (ring arithmetic).  None when the session
    is not a per-party one (the caller runs those steps)."""
    from moose_amd.parallel.spmd import Remote

    if not WSUM_FUSED or getattr(sess, "party_jobs", None) is None:
        return None
    ref = rows if rows is not None else x
    plc, bits = ref.plc, ref.bits
    if bits not in (64, 128):
        return None
    idx = sess.party_index(plc)
    nb = len(cblk)
    if idx is None:
        r = PV(plc, Remote(bits))
        t = RepTensor(plc, bits, "arith", r, r)
        return t if second is None or lead else (t, t)
    if rows is not None:
        k = len(weights)
        r0, r1 = rows.s0.v.data, rows.s1.v.data
        if not (r0.is_contiguous() and r1.is_contiguous()):
            return None
        per = tuple(r0.shape[1:-1] if bits == 128 else r0.shape[1:])
        r0, r1 = r0[:k], r1[:k]
    else:
        per = tuple(x.s0.v.data.shape[:-1] if bits == 128 else x.s0.v.data.shape)
        r0 = r1 = None
    L = max(1, math.prod(per))
    xs = None
    if x is not None:
        xs = (x.s0.v.data, x.s1.v.data)
    out = R.wsum_pair(bits, L, rows=None if r0 is None else (r0, r1), weights=weights, x=xs,
                      wx=wx, pub=(idx == 0, idx == 2), cblk=cblk, second=second,
                      like=(r0 if r0 is not None else xs[0]), lead=lead)
    if lead:
        nb += 1
    shp = ((nb * per[0],) + per[1:] if nb > 1 else per) + ((2,) if bits == 128 else ())
    o = RepTensor(plc, bits, "arith", PV(plc, R.RT(out[0].reshape(shp), bits)),
                  PV(plc, R.RT(out[1].reshape(shp), bits)))
    if second is None or lead:
        return o
    pshp = per + ((2,) if bits == 128 else ())
    return o, RepTensor(plc, bits, "arith", PV(plc, R.RT(out[2].reshape(pshp), bits)),
                        PV(plc, R.RT(out[3].reshape(pshp), bits)))


# MOOSEX_WSUM_FUSED=0: per-party local weighted sums as separate launches
WSUM_FUSED = os.environ.get("MOOSEX_WSUM_FUSED", "1") != "0"


def _rows_ok(sess, x) -> bool:
    """The session builds stacks in place and the mul kernel reads row views (device)."""
    return (getattr(sess, "p_rows_alloc", None) is not None and x.t.bits in (64, 128)
            and getattr(sess, "device", None) is not None and sess.device.type == "cuda")


def _poly_eval_rows(sess, x: RepFixed, coeffs, shift: int = 0) -> RepFixed:
    """poly_eval with the powers stack P preallocated: each level's multiplication reads
    x^h (a broadcast row) and P[0:m] (a slice) in place and its truncated product is
    written into rows h..h+m-1 -- the same protocol calls (and shares) as the generic
    path, without the per-level slice/concat copies."""
    n = len(coeffs) - 1
    f, bits, t = x.frac, x.bits, x.t
    pair = getattr(sess, "p_rows_alloc_pair", None)
    if pair is not None:
        P0, P1 = pair(t.s0, t.s1, n)
    else:
        P0, P1 = sess.p_rows_alloc(t.s0, n), sess.p_rows_alloc(t.s1, n)
    have = 1
    while have < n:
        m = min(2 * have, n) - have
        left = RepTensor(t.plc, bits, t.kind, sess.p_rows_bcast(P0, have - 1, m),
                         sess.p_rows_bcast(P1, have - 1, m))
        right = RepTensor(t.plc, bits, t.kind, sess.p_rows_view(P0, 0, m),
                          sess.p_rows_view(P1, 0, m))
        if getattr(sess, "fused", False):  # the trunc kernel writes rows have.. in place
            rep.mul_trunc(sess, left, right, f, out=(sess.p_rows_view(P0, have, have + m),
                                                     sess.p_rows_view(P1, have, have + m)))
        else:
            z = rep.trunc_pr(sess, rep.mul(sess, left, right), f)
            sess.p_rows_write(P0, have, z.s0)
            sess.p_rows_write(P1, have, z.s1)
        have += m
    P = RepTensor(t.plc, bits, t.kind, P0, P1)
    return _poly_tail(sess, P, coeffs, f, shift, x.integ)


def _batched_mul(sess, xs, ys):
    """Several independent fixed-point products in one round (stacked on a new axis)."""
    if len(xs) == 1:
        return [mul(sess, xs[0], ys[0])]
    X = concat(sess, [local(sess, v, "ExpandDims", axis=[0]) for v in xs], 0)
    Y = concat(sess, [local(sess, v, "ExpandDims", axis=[0]) for v in ys], 0)
    Z = mul(sess, X, Y)
    return [local(sess, Z, "IndexAxis", axis=0, index=i) for i in range(len(xs))]


@lru_cache(maxsize=None)
def _fit(fn_name: str, lo: float, hi: float, degree: int):
    """Least-squares Chebyshev fit -> monomial coefficients (float64)."""
    xs = np.cos(np.linspace(0, np.pi, 4001)) * (hi - lo) / 2 + (hi + lo) / 2
    fn = {
        "recip": lambda v: 1.0 / v,
        "sqrt": np.sqrt,
        "rsqrt": lambda v: 1.0 / np.sqrt(v),
        "log2": np.log2,
        "exp2": np.exp2,
    }[fn_name]
    poly = np.polynomial.Polynomial.fit(xs, fn(xs), degree).convert()
    return tuple(float(c) for c in poly.coef)


# ---------------------------------------------------------------------------
# reciprocal / division / sqrt / log
# ---------------------------------------------------------------------------
def _newton_recip(sess, m: RepFixed, w: RepFixed, iters: int) -> RepFixed:
    for _ in range(iters):
        e = const_sub(sess, 2.0, mul(sess, m, w))  # 2 - m w
        w = mul(sess, w, e)
    return w


def reciprocal_positive(sess, x: RepFixed) -> RepFixed:
    m, t, lo, hi = _normalize(sess, x)
    f = x.frac
    w = poly_eval(sess, m, _fit("recip", 0.5, 1.0, 4))
    w = _newton_recip(sess, m, w, 2 if f > 24 else 1)
    weights = [(1 << (2 * f - 1 - j)) if 2 * f - 1 - j >= 0 else 0 for j in range(lo, hi)]
    F = RepFixed(_weighted(sess, t, weights, x.bits), f, x.integ)
    return mul(sess, w, F)


def reciprocal(sess, x: RepFixed) -> RepFixed:
    s = sign_bit(sess, x)
    ax = _with(x, rep.negate_where(sess, s, x.t))
    r = reciprocal_positive(sess, ax)
    return _with(r, rep.lincomb(sess, [(1, r.t), (-2, rep.mul(sess, s, r.t))]))


def div(sess, x, y, px=None, py=None):
    if py is not None:
        # public divisor: multiply by its reciprocal computed in the clear
        yv = R.decode(_pub(py), x.frac)
        inv = R.encode(1.0 / yv, x.frac, x.bits)
        return _with(x, rep.trunc_pr(sess, rep.mul_public(sess, x.t, inv), x.frac))
    r = reciprocal(sess, y)
    if px is not None:
        return _with(r, rep.trunc_pr(sess, rep.mul_public(sess, r.t, _pub(px)), r.frac))
    return mul(sess, x, r)


def sqrt(sess, x: RepFixed) -> RepFixed:
    """sqrt(x) = sqrt(m) * 2^((j - f + 1) / 2) for x = m * 2^(j-f+1), m in [0.5, 1)."""
    m, t, lo, hi = _normalize(sess, x)
    f = x.frac
    sm = poly_eval(sess, m, _fit("sqrt", 0.5, 1.0, 5))
    weights = [int(round(2.0 ** ((j - f + 1) / 2.0) * (1 << f))) for j in range(lo, hi)]
    G = RepFixed(_weighted(sess, t, weights, x.bits), f, x.integ)
    return mul(sess, sm, G)


def log2(sess, x: RepFixed) -> RepFixed:
    """log2(x) = log2(m) + (j - f + 1)."""
    m, t, lo, hi = _normalize(sess, x)
    f = x.frac
    lm = poly_eval(sess, m, _fit("log2", 0.5, 1.0, 8))
    weights = [((j - f + 1) << f) for j in range(lo, hi)]
    E = _weighted(sess, t, weights, x.bits)
    return _with(lm, rep.add(sess, lm.t, E))


def log(sess, x: RepFixed) -> RepFixed:
    return mul_const(sess, log2(sess, x), math.log(2.0))


# ---------------------------------------------------------------------------
# exponentials
# ---------------------------------------------------------------------------
def _exp2_parts(sess, a: RepFixed, negative: bool):
    """2^a (or 2^-a) for a >= 0: integer part from B2A'd bits (product tree of public
    factors), fraction via polynomial."""
    f, bits, integ = a.frac, a.bits, a.integ
    # every integer bit of a must be inspected (a < 2^(integ+1) after the log2(e) scale)
    nint = max(1, min(bits - 2 - f, integ + 1))
    # the product tree below runs over a power-of-two number of factors: extra factors are
    # exactly 1 (bit planes above the integer range with weight 0), so no level has an odd
    # factor to carry over (a slice + concat per party vector per odd level otherwise)
    npad = 1 << (nint - 1).bit_length()
    if f + npad > bits:
        npad = nint
    # parties on different processes (rounds cost messages): the polynomial and the
    # product tree advance together (_merged_exp_tail)
    merged = (negative and not getattr(sess, "is_simulated", True)
              and getattr(sess, "party_dot_trunc", None) is not None
              and hasattr(sess, "p_cross_plain") and npad >= 2 and npad & (npad - 1) == 0)
    # only bits below f + nint are read with a nonzero weight (higher planes are padding
    # whose factor is 1 whatever the bit): the adder need not carry beyond them
    # (bounded by construction, unlike a sign: planes above f + nint are never read, so a
    # carry into them cannot change the result)
    bd = rep.bit_decompose(sess, a.t, width=f + nint if EXP_WIDTH and f + nint < bits else None)
    ab = rep.b2a_planes(sess, bd, 0, f + npad, bits)  # arithmetic bits, leading axis
    return _exp2_from_planes(sess, ab, f, integ, bits, nint, npad, negative, merged)


def _exp2_from_planes(sess, ab: RepTensor, f: int, integ: int, bits: int, nint: int,
                      npad: int, negative: bool, merged: bool, cs=None,
                      plus: float = 0.0) -> RepFixed:
    """2^a (2^-a) from the arithmetic bit planes ``ab`` of a >= 0 at ``f`` fractional bits:
    rows 0..f-1 the fraction, rows f..f+npad-1 the integer part (rows from nint on weigh 0).
    ``cs``: the factor rows' public weights (c_j - 1) 2^f when the caller chose them.
    ``plus``: a public constant added to the result (in the last product's tail when the
    batched per-party tail runs it, else one add)."""
    frac_w = [(1 << j) for j in range(f)] + [0] * npad
    fused = _wsum(sess, ab, [-(1 << j) for j in range(f)], cblk=(1 << f,)) if negative else None
    if fused is not None:  # 1 - r in one launch (weighted sum, negation, public 1)
        px, shift = RepFixed(fused, f, integ), 1
    elif negative:
        r = RepFixed(_weighted(sess, ab, frac_w, bits), f, integ)
        # 2^-r for r in [0,1) = 2^(1-r) / 2 -> fit exp2 on [0, 1] of (1 - r)
        px, shift = const_sub(sess, 1.0, r), 1
    else:
        px, shift = RepFixed(_weighted(sess, ab, frac_w, bits), f, integ), 0
    one_minus = px
    # integer part factors 1 + b_j (c_j - 1), c_j = 2^(+-2^j), for all j at once: the
    # integer bit planes stay stacked on the leading axis, scaled by a public vector
    cs = [] if cs is None else list(cs)
    for j in range(nint if not cs else 0):
        e = 2 ** j
        if negative:
            c = 2.0 ** (-e) if e <= f + 2 else 0.0  # underflows to 0 at precision f
        else:
            c = 2.0 ** min(e, integ + 1)  # saturate: larger results overflow anyway
        cs.append(int(round((c - 1.0) * (1 << f))))
    cs += [0] * (npad - nint)
    ints = local(sess, ab, "Slice", slice=(f, f + npad, None))
    cvec = R.const_ints(cs, bits, sess.device)
    one = _encode_const(sess, 1.0, f, bits)
    both = getattr(sess, "p_mul_leading_add", None)
    r = both(ints.plc, ints.s0, ints.s1, cvec, one) if both is not None else None
    if r is not None:  # the two steps below in one launch (same values)
        fac = RepTensor(ints.plc, bits, "arith", r[0], r[1])
    else:
        pc = sess.public(ints.plc, cvec)
        fac = RepTensor(ints.plc, bits, "arith", *rep._sharewise(
            sess, "MulLeading", ints.plc, (ints.s0, ints.s1), (pc, pc)))
        fac = rep.add_public(sess, fac, one)
    if merged:
        # parties on different processes: the polynomial's levels and the product tree's
        # levels are independent -- each round carries both (module doc: _merged_exp_tail)
        return _merged_exp_tail(sess, one_minus, fac, npad, plus=plus)
    # the polynomial's power levels and the product tree's levels (a log-depth product over
    # the leading axis) advance together: each round's two products run as one launch on a
    # stacked device session (rep.mul_trunc_many)
    p, F = _poly_and_tree(sess, px, _fit("exp2", 0.0, 1.0, 7), shift,
                          RepFixed(fac, f, integ), npad)
    e = mul(sess, p, local(sess, F, "IndexAxis", axis=0, index=0))
    return add_const(sess, e, plus) if plus else e


def _poly_and_tree(sess, x: RepFixed, coeffs, shift: int, F: RepFixed, nf: int):
    """(poly_eval(x, coeffs, shift), the product of F's ``nf`` leading entries as a
    1-entry stack) with one level of each per round: the polynomial's powers x^(h+1..h+m)
    = x^h * P[0:m] (in place in a row stack on a stacked device session, else by slice /
    concat) and the tree's F[0:h] * F[h:2h].  Same values as the two computed one after
    the other."""
    n = len(coeffs) - 1
    f, bits, t = x.frac, x.bits, x.t
    rows = n > 1 and _rows_ok(sess, x)
    views = _rows_ok(sess, F)
    if rows:
        pair = getattr(sess, "p_rows_alloc_pair", None)
        P0, P1 = pair(t.s0, t.s1, n) if pair is not None else (
            sess.p_rows_alloc(t.s0, n), sess.p_rows_alloc(t.s1, n))
    else:
        P = local(sess, x, "ExpandDims", axis=[0])
    have = 1
    while have < n or nf > 1:
        jobs = []
        m = min(2 * have, n) - have if have < n else 0
        if m:
            if rows:
                left = RepTensor(t.plc, bits, t.kind, sess.p_rows_bcast(P0, have - 1, m),
                                 sess.p_rows_bcast(P1, have - 1, m))
                right = RepTensor(t.plc, bits, t.kind, sess.p_rows_view(P0, 0, m),
                                  sess.p_rows_view(P1, 0, m))
                out = (sess.p_rows_view(P0, have, have + m), sess.p_rows_view(P1, have, have + m))
                jobs.append((left, right, f, out))
            else:
                xh = local(sess, P, "Slice", slice=(have - 1, have, None))
                left = xh if m == 1 else concat(sess, [xh] * m, 0)
                right = P if m == have else local(sess, P, "Slice", slice=(0, m, None))
                jobs.append((left.t, right.t, f, None))
        h = nf // 2
        if h:
            if views:  # both halves read in place by the mul kernel
                lo = RepTensor(F.t.plc, bits, "arith", sess.p_rows_view(F.t.s0, 0, h),
                               sess.p_rows_view(F.t.s1, 0, h))
                hi = RepTensor(F.t.plc, bits, "arith", sess.p_rows_view(F.t.s0, h, 2 * h),
                               sess.p_rows_view(F.t.s1, h, 2 * h))
            else:
                lo = local(sess, F.t, "Slice", slice=(0, h, None))
                hi = local(sess, F.t, "Slice", slice=(h, 2 * h, None))
            jobs.append((lo, hi, F.frac, None))
        if rows and m and not getattr(sess, "fused", False):
            # the unfused rows path writes the level's rows itself (as _poly_eval_rows)
            z = rep.trunc_pr(sess, rep.mul(sess, jobs[0][0], jobs[0][1]), f)
            sess.p_rows_write(P0, have, z.s0)
            sess.p_rows_write(P1, have, z.s1)
            res = [None] + rep.mul_trunc_many(sess, jobs[1:])
        else:
            res = rep.mul_trunc_many(sess, jobs)
        k = 0
        if m:
            if not rows:
                P = concat(sess, [P, _with(x, res[0])], 0)
            have += m
            k = 1
        if h:
            prod = _with(F, res[k])
            F = prod if nf % 2 == 0 else concat(
                sess, [prod, local(sess, F, "Slice", slice=(2 * h, nf, None))], 0)
            nf = (nf + 1) // 2
    Pt = RepTensor(t.plc, bits, t.kind, P0, P1) if rows else P.t
    if n <= 1:
        Pt = local(sess, x, "ExpandDims", axis=[0]).t
    return _poly_tail(sess, Pt, coeffs, f, shift, x.integ), F


def _poly_tail(sess, Pt: RepTensor, coeffs, f: int, shift: int, integ: int) -> RepFixed:
    """sum_k c_k P[k-1] truncated by f + shift, plus c_0 / 2^shift: one launch on a stacked
    device session (p_wsum_trunc_add), else weighted sum + TruncPr + add (same shares)."""
    bits = Pt.bits
    weights = [int(round(c * (1 << f))) for c in coeffs[1:]]
    c0 = coeffs[0] / (1 << shift)
    fused = getattr(sess, "p_wsum_trunc_add", None)
    if fused is not None and getattr(sess, "fused", False):
        r = fused(Pt.plc, Pt.s0, weights, f + shift, int(round(c0 * (1 << f))))
        if r is not None:
            return RepFixed(RepTensor(Pt.plc, bits, "arith", r[0], r[1]), f, integ)
    acc = _weighted(sess, Pt, weights, bits)
    acc = rep.trunc_pr(sess, acc, f + shift)
    return add_const(sess, RepFixed(acc, f, integ), c0)


def _tail_trunc(sess, plc, v, bits, m) -> RepTensor:
    """Zero share + reshare + TruncPr(m) of local 3-out-of-3 additive products ``v`` (a
    party vector): the dot's tail (parallel/party.py); 2 rounds."""
    nonces = tuple(sess.nonce(plc) for _ in range(7))
    s0, s1 = sess.party_dot_trunc(plc, v, m, nonces)
    return RepTensor(plc, bits, "arith", s0, s1)


def _merged_exp_tail(sess, x: RepFixed, fac: RepTensor, npad: int,
                     plus: float = 0.0) -> RepFixed:
    """2^-a = p(1 - r) / 2 * prod(factors) with the polynomial p (degree 7) and the
    product tree over the ``npad`` integer-bit factors evaluated TOGETHER: every round's
    messages carry one level of each -- the level's products are ONE batched tail (local
    cross terms concatenated on the stacking axis, one zero share + reshare + TruncPr) --
    and the polynomial's final TruncPr (its terms' additive shares) rides with a tree level
    too.  For the tutorial LR (fixed(24,40): 32 factors) 20 rounds become 12; the values
    are those of poly_eval + the tree up to TruncPr's probabilistic rounding."""
    if _jobs_ok(sess, x.t, fac):
        return _merged_exp_tail_jobs(sess, x, fac, npad, plus=plus)
    coeffs = _fit("exp2", 0.0, 1.0, 7)
    f, bits, t = x.frac, x.bits, x.t
    plc = t.plc
    n = len(coeffs) - 1
    ex = lambda v: local(sess, v, "ExpandDims", axis=[0])  # noqa: E731

    def sl(v, a, b):
        return local(sess, v, "Slice", slice=(a, b, None))

    def run(pairs, truncs=()):
        """One round: the products of ``pairs`` (stacked operands) and the TruncPr of the
        first-share vectors ``truncs``, as one tail; returns the pieces in order."""
        parts, sizes = [], []
        for a, b in pairs:
            parts.append(sess.p_cross_plain("arith", plc, a.s0, a.s1, b.s0, b.s1))
            sizes.append(sess.p_shape(a.s0)[0])
        for v in truncs:
            parts.append(v)
            sizes.append(sess.p_shape(v)[0])
        v = parts[0] if len(parts) == 1 else sess.p("Concat", plc, *parts, axis=0)
        out = _tail_trunc(sess, plc, v, bits, f)
        res, at = [], 0
        for k in sizes:
            res.append(out if len(sizes) == 1 else sl(out, at, at + k))
            at += k
        return res

    P = ex(t)          # powers of x, stacked: [x, x^2, ...]
    F = fac            # tree factors, stacked
    have, nf = 1, npad
    while have < n:  # one polynomial level + one tree level per round
        m = min(2 * have, n) - have
        xh = sl(P, have - 1, have)
        left = xh if m == 1 else concat(sess, [xh] * m, 0)
        right = P if m == have else sl(P, 0, m)
        pairs = [(left, right)]
        if nf > 1:
            pairs.append((sl(F, 0, nf // 2), sl(F, nf // 2, nf)))
        got = run(pairs)
        P = concat(sess, [P, got[0]], 0)
        if nf > 1:
            F, nf = got[1], nf // 2
        have += m
    # the polynomial's weighted sum (local) and its TruncPr ride with the next tree level
    acc = _weighted(sess, P, [int(round(c * (1 << f))) for c in coeffs[1:]], bits)
    acc_v = ex(acc).s0  # party p's first share: a 3-out-of-3 additive sharing of acc
    if nf > 1:
        F, acc_t = run([(sl(F, 0, nf // 2), sl(F, nf // 2, nf))], [acc_v])
        nf //= 2
    else:
        acc_t = run([], [acc_v])[0]
    p = add_const(sess, RepFixed(local(sess, acc_t, "IndexAxis", axis=0, index=0), f, x.integ),
                  coeffs[0])
    while nf > 1:
        F, nf = run([(sl(F, 0, nf // 2), sl(F, nf // 2, nf))])[0], nf // 2
    # 2^-a = p(1 - r) / 2 * prod: the halving is one more bit of the last TruncPr
    e = mul(sess, p, RepFixed(local(sess, F, "IndexAxis", axis=0, index=0), f, x.integ),
            f=f + 1)
    return add_const(sess, e, plus) if plus else e


def _jobs_ok(sess, *reps) -> bool:
    """A per-party session whose products can run through the batched tail kernels
    (csrc/rss_jobs.hip): same-shape dense shares within each operand (a pending dot is
    judged by its additive share, without completing it)."""
    if getattr(sess, "party_jobs", None) is None or not rep.JOBS:
        return False
    if os.environ.get("MOOSEX_DOT_TAIL", "1") == "0" or reps[0].bits not in (64, 128):
        return False
    if sess.party_index(reps[0].plc) is None:
        return True

    def ok(r):
        if isinstance(r, rep.PendingTrunc) and not r.completed:
            return isinstance(r.v_add, R.RT) and r.v_add.data.is_contiguous()
        return all(isinstance(t.v, R.RT) and t.v.data.is_contiguous()
                   and t.v.shape == r.s0.v.shape for t in (r.s0, r.s1))
    return all(ok(r) for r in reps)


def _abs_scaled_jobs(sess, s: RepTensor, x: RepFixed, c: float) -> RepFixed:
    """|x| * c (one truncation) on a per-party session, for the arithmetic sign bit s of x:
    trunc(c x - 2 c s x) -- the product s x, the public scaling and the truncation in ONE
    batched tail (job value c x_p - 2c cross(s, x)_p): 2 rounds and 3 kernels instead of
    negate_where's multiplication round plus mul_const's TruncPr (3 rounds, ~7 kernels)."""
    cv = int(round(c * (1 << x.frac)))
    t = x.t
    nonces = _tail_nonces(sess, t.plc)
    r = rep.tail_job(sess, t.plc, t.bits, x.frac, nonces, t.s0,
                     lambda o0, o1: R.MulJob(1, o0, o1, x=(s.s0.v.data, s.s1.v.data),
                                             y=(t.s0.v.data, t.s1.v.data), cb=-2 * cv,
                                             a=t.s0.v.data, ca=cv))
    return _with(x, r)


class _Stack:
    """A party's rows for the batched tails: ``x`` (the first power, its own tensors) and
    a dense [k, ...] stack per share component for the rows after it."""

    def __init__(self, x0, x1, rows, bits):
        self.x0, self.x1, self.bits = x0, x1, bits
        shp = (rows,) + tuple(x0.shape)
        self.s0 = torch.empty(shp, dtype=x0.dtype, device=x0.device)
        self.s1 = torch.empty(shp, dtype=x0.dtype, device=x0.device)

    def power(self, k):
        """(share0, share1) tensors of x^k (k >= 1)."""
        return (self.x0, self.x1) if k == 1 else (self.s0[k - 2], self.s1[k - 2])


def _power_jobs(st: _Stack, have: int, m: int, L: int):
    """Jobs of one power level: x^(have+1 .. have+m) = x^have * [x, x^2, .., x^m], written
    into the stack rows (as the generic level's concat of x^have copies times P[0:m])."""
    left = st.power(have)
    jobs = [R.MulJob(1, st.s0[have - 1], st.s1[have - 1], x=left, y=st.power(1))]
    if m > 1:
        jobs.append(R.MulJob(m - 1, st.s0[have:have + m - 1], st.s1[have:have + m - 1], x=left,
                             y=(st.s0[0], st.s1[0]), sx=0, sy=L))
    return jobs


def _acc_job(st: _Stack, weights, n, L, o0, o1):
    """The additive share sum_k w_k x^k (this party's first share components) as a value
    job: the stack rows by one weighted-sum kernel, x^1 as the job's second term."""
    rest = R.weighted_sum(R.RT(st.s0[:n - 1], st.bits), [w % (1 << st.bits) for w in weights[1:n]])
    return R.MulJob(1, o0, o1, a=rest.data, sa=L, a2=st.x0, sa2=L, ca2=weights[0])


def _tail_nonces(sess, plc):
    return tuple(sess.nonce(plc) for _ in range(7))


def _merged_exp_tail_jobs(sess, x: RepFixed, fac: RepTensor, npad: int,
                          plus: float = 0.0) -> RepFixed:
    """_merged_exp_tail on the batched per-party tail (csrc/rss_jobs.hip): every round is the
    tail's three kernels for all of that round's products -- the polynomial level's (read
    from and written into a preallocated power stack), the tree level's, and the
    polynomial's weighted sum when it rides along -- with the same nonces, the same element
    order and so bitwise the same shares as the generic rounds (cross terms per pair,
    concatenation, tail, slices)."""
    from moose_amd.parallel.spmd import Remote

    coeffs = _fit("exp2", 0.0, 1.0, 7)
    f, bits, t = x.frac, x.bits, x.t
    plc = t.plc
    n = len(coeffs) - 1
    weights = [int(round(c * (1 << f))) for c in coeffs[1:]]
    member = sess.party_index(plc) is not None
    shape = sess.p_shape(t.s0) if member else None
    L = max(1, math.prod(shape)) if member else 1
    st = _Stack(t.s0.v.data, t.s1.v.data, n - 1, bits) if member else None
    F0, F1 = (fac.s0.v.data, fac.s1.v.data) if member else (None, None)

    def run(jobs, m=f, defer=False):
        nonces = _tail_nonces(sess, plc)
        if member:
            sess.party_jobs(plc, jobs, L, bits, m, nonces, defer=defer)

    def tree_job(nf):
        h = nf // 2
        o0 = torch.empty_like(F0[0:h])
        o1 = torch.empty_like(F0[0:h])
        return R.MulJob(h, o0, o1, x=(F0[0:h], F1[0:h]), y=(F0[h:2 * h], F1[h:2 * h]), sx=L,
                        sy=L), (o0, o1)

    have, nf = 1, npad
    while have < n:  # one polynomial level + one tree level per round
        m = min(2 * have, n) - have
        jobs = _power_jobs(st, have, m, L) if member else []
        new = None
        if nf > 1 and member:
            tj, new = tree_job(nf)
            jobs.append(tj)
        run(jobs, defer=True)  # its round-2 sums ride in the next level's round 0
        if nf > 1:
            F0, F1 = new if member else (None, None)
            nf //= 2
        have += m
    if member:
        sess.party_jobs_flush(plc)  # the power stack and the tree rows, before other reads
    fw = 62 - f  # the polynomial's weights' fractional bits in the one-product finish
    if EXP_ONE_PRODUCT and nf == 1 and bits == 128 and fw >= 20:
        # the tree is done with the powers: e = p F / 2 as ONE product -- the polynomial's
        # weighted sum ACC = sum_k w_k x^k (w_k at fw bits) is a local combination of the
        # replicated powers, so cross(ACC, F) + c_0 2^(f+fw) F_first is an additive share
        # of p F at scale 2^(2f+fw), truncated by f + fw + 1 = 63 bits in the same tail
        # (instead of the weighted sum's TruncPr round pair, then the product's)
        wts = [int(round(c * (1 << fw))) for c in coeffs[1:]]
        c0 = int(round(coeffs[0] * (1 << (f + fw))))
        if member:
            mod = 1 << bits
            if WSUM_FUSED:  # both components' sums in one launch
                L = max(1, math.prod(shape))
                a0, a1 = R.wsum_pair(bits, L, rows=(st.s0[:n - 1], st.s1[:n - 1]),
                                     weights=wts[1:], x=(st.x0, st.x1), wx=wts[0],
                                     pub=(False, False))
                acc = [a0.reshape(st.x0.shape), a1.reshape(st.x0.shape)]
            else:
                acc = []
                for X, rows in ((st.x0, st.s0), (st.x1, st.s1)):
                    rest = R.weighted_sum(R.RT(rows[:n - 1], bits), [w % mod for w in wts[1:]])
                    lin = R.binary("mul", R.RT(X, bits), R.fill((), wts[0], bits, X.device))
                    acc.append(R.binary("add", rest, lin).data)
            o0, o1 = torch.empty_like(st.x0), torch.empty_like(st.x0)
            # the public ``plus`` rides in the tail: party 0 adds it at the product's
            # untruncated scale (a multiple of 2^m: the truncation carries it exactly)
            pk = int(round(plus * (1 << f))) << (f + fw + 1) if PLUS_IN_TAIL else 0
            a2 = (R.const_ints([pk % mod] * L, bits, st.x0.device).data
                  if pk and sess.party_index(plc) == 0 else None)
            run([R.MulJob(1, o0, o1, x=(acc[0], acc[1]), y=(F0[0], F1[0]), a=F0[0], ca=c0,
                          a2=a2)], m=f + fw + 1)
            e = RepTensor(plc, bits, "arith", PV(plc, R.RT(o0, bits)), PV(plc, R.RT(o1, bits)))
        else:
            run([], m=f + fw + 1)
            r = PV(plc, Remote(bits))
            e = RepTensor(plc, bits, "arith", r, r)
        e = RepFixed(e, f, x.integ)
        return add_const(sess, e, plus) if plus and not PLUS_IN_TAIL else e
    # the polynomial's weighted sum rides with the next tree level (its TruncPr)
    acc0 = acc1 = None
    jobs = []
    new = None
    if member and nf > 1:
        tj, new = tree_job(nf)
        jobs.append(tj)
    if member:
        acc0, acc1 = torch.empty_like(st.x0), torch.empty_like(st.x0)
        jobs.append(_acc_job(st, weights, n, L, acc0, acc1))
    run(jobs)
    if nf > 1:
        F0, F1 = new if member else (None, None)
        nf //= 2
    while nf > 1:
        new = None
        if member:
            tj, new = tree_job(nf)
            run([tj])
        else:
            run([])
        F0, F1 = new if member else (None, None)
        nf //= 2
    if not member:
        r = PV(plc, Remote(bits))
        acc = RepTensor(plc, bits, "arith", r, r)
        F = acc
    else:
        acc = RepTensor(plc, bits, "arith", PV(plc, R.RT(acc0, bits)), PV(plc, R.RT(acc1, bits)))
        F = RepTensor(plc, bits, "arith", PV(plc, R.RT(F0[0], bits)), PV(plc, R.RT(F1[0], bits)))
    p = add_const(sess, RepFixed(acc, f, x.integ), coeffs[0])
    # 2^-a = p(1 - r) / 2 * prod: the halving is one more bit of the last TruncPr
    e = mul(sess, p, RepFixed(F, f, x.integ), f=f + 1)
    return add_const(sess, e, plus) if plus else e


def exp2(sess, x: RepFixed) -> RepFixed:
    s = sign_bit(sess, x)
    ax = _with(x, rep.negate_where(sess, s, x.t))
    pos = _exp2_parts(sess, ax, negative=False)
    negv = _exp2_parts(sess, ax, negative=True)
    return _with(pos, rep.mux(sess, s, negv.t, pos.t))


def exp(sess, x: RepFixed) -> RepFixed:
    return exp2(sess, mul_const(sess, x, 1.0 / math.log(2.0)))


def exp_nonpositive(sess, x: RepFixed) -> RepFixed:
    """e^x for x <= 0 (softmax after max subtraction, sigmoid): no sign mux."""
    a = mul_const(sess, neg(sess, x), 1.0 / math.log(2.0))
    return _exp2_parts(sess, a, negative=True)


def sigmoid(sess, x: RepFixed) -> RepFixed:
    """sigma(x) = 1 / (1 + e^-|x|) mirrored for x < 0; 1 + e^-|x| is in [1, 2] so the
    reciprocal needs no normalisation."""
    # (s, 1 + e^-|x|): the 1 rides in the exp's last tail
    one = _sign_and_exp_party(sess, x, plus=1.0) if _jobs_ok(sess, x.t) else None
    if one is not None:
        s, d = one
        party = True
    else:
        s = sign_bit(sess, x)
        party = _jobs_ok(sess, x.t, s)
    if one is not None:
        pass
    elif party:
        # per-party: |x| / ln 2 in one tail (_abs_scaled_jobs), one round fewer
        e = _exp2_parts(sess, _abs_scaled_jobs(sess, s, x, 1.0 / math.log(2.0)), negative=True)
    else:
        ax = _with(x, rep.negate_where(sess, s, x.t))
        e = exp_nonpositive(sess, neg(sess, ax))
    if one is None:
        d = add_const(sess, e, 1.0)  # in [1, 2]
    # 1/d = (1/h) / 2 with h = d / 2 in [0.5, 1]: the fit of 1/h evaluated at d directly
    # (coefficients c_k / 2^k), and both halvings folded into TruncPrs of one more bit --
    # no round spent on multiplying by 0.5
    if party and RECIP_DIRECT and d.frac >= 36:
        # one party per process (rounds cost messages): a degree-8 fit of 1/h (max error
        # 4.4e-7 on [0.5, 1], 2.2e-7 on the probability) has three power levels -- 8 rounds
        # instead of 10 for the degree-4 fit and its Newton step.  Its coefficients alternate
        # up to ~700 (sum of magnitudes ~2600), so it needs the fractional bits to absorb that
        # cancellation: below 36 the Newton form is more accurate
        coeffs = tuple(c / (1 << k) for k, c in enumerate(_fit("recip", 0.5, 1.0, 8)))
        f, bits = d.frac, d.bits
        if DEFER_OUTPUT_TRUNC and _jobs_ok(sess, d.t) and 2 * f + 16 < bits:
            # the polynomial's weighted sum W = sum_k w_k d^k is a LOCAL combination of the
            # replicated powers (scale 2^2f), so pos * 2^(2f+1) = W + c_0 2^2f needs no
            # round; sigma * 2^(2f+1) = pos' + s (2^(2f+1) - 2 pos') is one mul_add whose
            # reshare AND truncation by f + 1 wait for the reader -- the reveal opens it in
            # one round and shifts exactly (2 rounds fewer than TruncPr(W) then mul_add)
            c0 = int(round(coeffs[0] * (1 << (2 * f))))
            big, diff = _poly_powers_sum(sess, d, coeffs,
                                         finish=(c0, -2, int(round(1.0 * (1 << (2 * f + 1))))))
            return RepFixed(rep.mul_add_trunc(sess, s, diff, big, f + 1), f, d.integ)
        pos = poly_eval(sess, d, coeffs, shift=1)
    else:
        w = poly_eval(sess, d, tuple(c / (1 << k)
                                     for k, c in enumerate(_fit("recip", 0.5, 1.0, 4))))
        hw = mul(sess, d, w, f=d.frac + 1)  # h w
        pos = mul(sess, w, const_sub(sess, 2.0, hw), f=w.frac + 1)  # one Newton step, halved
    if party:
        # sigma = pos + s (1 - 2 pos); the product's reshare waits for the reader (a reveal
        # absorbs it: parallel/party.py MulAddTail)
        diff = rep.lincomb(sess, [(-2, pos.t)], const=_encode_const(sess, 1.0, pos.frac,
                                                                      pos.bits))
        return _with(pos, rep.mul_add(sess, s, diff, pos.t))
    one_minus = const_sub(sess, 1.0, pos)
    return _with(pos, rep.mux(sess, s, one_minus.t, pos.t))


# per-party sessions leave a public-operand dot's TruncPr pending until it is read
DEFER_DOT_TRUNC = os.environ.get("MOOSEX_DEFER_DOT_TRUNC", "1") != "0"
# ... and add a public constant after it (the sigmoid's 1 + e^-|x|) inside its tail
PLUS_IN_TAIL = True
# per-party sessions finish 2^-a with one product (the polynomial's sum untruncated)
EXP_ONE_PRODUCT = os.environ.get("MOOSEX_EXP_ONE_PRODUCT", "1") != "0"
# per-party sessions evaluate the sigmoid's reciprocal as one degree-8 polynomial
RECIP_DIRECT = os.environ.get("MOOSEX_RECIP_DIRECT", "1") != "0"
# per-party sessions leave the sigmoid's last truncation to its reader (a reveal: exact)
DEFER_OUTPUT_TRUNC = os.environ.get("MOOSEX_SIGMOID_DEFER_TRUNC", "1") != "0"
# per-party sessions take the sigmoid's sign and e^-|x| from one bit decomposition
ONE_DECOMPOSITION = os.environ.get("MOOSEX_SIGMOID_ONE_BITDEC", "1") != "0"
# ... with the integer bits whose factor underflows replaced by a range check (3 blocks)
RANGE_SPLIT = os.environ.get("MOOSEX_EXP_RANGE_SPLIT", "1") != "0"

def _sign_and_exp_party(sess, x: RepFixed, plus: float = 0.0):
    """(s, e^-|x|) for a per-party session from ONE bit decomposition: z = x * C with C =
    log2(e) at ``fc`` fractional bits is a LOCAL product (no truncation: z keeps F = f + fc
    fractional bits, |z| < 2^(integ + 1 + F)); its planes XORed with its sign plane are the
    planes of |z| (up to one unit of z's last bit: ~z = -z - 1), so one adder gives the sign
    s (arithmetic, for the final mirror) and, from plane F - f on, |z| floored to f
    fractional bits -- the input of 2^-a (_exp2_from_planes).  Replaces the sign's
    decomposition, the |x| / ln 2 tail and the second decomposition (8 + 2 + 8 rounds become
    9 for the tutorial LR).  The floor differs from TruncPr's rounding by < 2^-f.

    Only the integer bits j with a factor 2^-(2^j) that does not underflow at f bits
    (2^j <= f + 2: jn of them) are factors of their own; |z| >= T = 2^(F + jn) makes e^-|x|
    < 2^-(2^jn), zero at f bits, so the bits above are replaced by [z >= T] and [z < -T]:
    the sign planes of x - T' and x + T' (T' = T / C), decomposed in the SAME adder (the
    blocks z, x - T', x + T', x; same rounds).  The mirror's sign and the range flags are
    the ring's msb of x's blocks, so they are right for every representable x, not only
    below the type's nominal 2^integ.  Their factors 1 - [z >= T] and 1 - [z < -T] join the tree: jn + 2 factors
    (8 for fixed(24, 40)) instead of 25 -> 32, two tree levels (4 rounds) fewer.
    None when the ring has too few bits for fc >= 20 (the caller uses the three steps)."""
    if not ONE_DECOMPOSITION or getattr(sess, "is_simulated", True):
        return None
    f, integ, bits = x.frac, x.integ, x.bits
    # a dot whose TruncPr is pending (rep.PendingTrunc): decompose its untruncated value
    # (m more fractional bits) after ONE reshare round instead of the tail's two
    pend = x.t if isinstance(x.t, rep.PendingTrunc) and not x.t.completed else None
    extra = pend.m if pend is not None else 0
    fc = min(f, bits - 3 - integ - f - extra)
    if fc < 20 and pend is not None:
        pend, extra = None, 0  # too few ring bits for both: complete the dot first
        fc = min(f, bits - 3 - integ - f)
    if fc < 20:
        return None
    F = f + extra + fc
    q = integ + 1 + F  # the sign plane: |z| < 2^(q)
    nint = max(1, min(bits - 2 - f, integ + 1))
    if q > bits - 1 or F + nint > q:
        return None
    jn = 1
    while jn < nint and (1 << jn) <= f + 2:
        jn += 1
    split = RANGE_SPLIT and jn < nint and F + jn < q
    if pend is not None and not split and F + (1 << (nint - 1).bit_length()) > bits:
        # the full product tree's planes would not fit above the pending scale: complete
        # the dot first (the tail's two rounds) and decompose at the type's scale
        pend = None
        F -= extra
        q -= extra
    C = int(round(math.log2(math.e) * (1 << fc)))
    xt = pend.reshare_untruncated() if pend is not None else x.t
    fx = f + (pend.m if pend is not None else 0)  # x' = xt's fractional bits
    if split:
        # blocks z, x' - T', x' + T', x' (T' = T / C in x's units): |z|'s planes come from
        # z (plane q its sign), but the range flags and the mirror's sign come from x' at the
        # ring's msb -- right for every representable x, not only |x| < 2^integ (a product
        # keeps the nominal integ while its value grows)
        Tv = 1 << (F + jn)
        Tx = -(-Tv // C)  # z >= T  <=>  x' >= Tx (x' an integer at fx bits)
        # the four blocks in one launch (z = C x' as block 0), no concatenation
        zs = _wsum(sess, None, (), x=xt, wx=1, cblk=(-Tx, Tx, 0), second=(C, 0), lead=True)
        if zs is None:
            z = rep.lincomb(sess, [(C, xt)])
            T = R.fill((), Tx, bits, sess.device)
            xs = concat(sess, [RepFixed(rep.sub_public(sess, xt, T), fx, integ),
                               RepFixed(rep.add_public(sess, xt, T), fx, integ),
                               RepFixed(xt, fx, integ)], 0).t
            zs = concat(sess, [RepFixed(z, F, integ), RepFixed(xs, fx, integ)], 0).t
        nfac = jn + 2
        npad = 1 << (nfac - 1).bit_length()
        extra = npad - nfac  # planes above jn whose factor is 1 (weight 0)
        bd = rep.bit_decompose(sess, zs)  # all bits: the signs are the ring's msb
        ab = rep.b2a_planes_xor(sess, bd, F - f, f + jn + extra, q, bits, blocks=4,
                                sbit=bits - 1)
        cs = []
        for j in range(jn):
            cs.append(int(round((2.0 ** -(2 ** j) - 1.0) * (1 << f))))
        cs += [0] * extra + [-(1 << f)] * 2  # the range factors 1 - b
        rows = local(sess, ab, "Slice", slice=(0, f + npad, None))
        s = local(sess, ab, "IndexAxis", axis=0, index=f + npad)
        nint_used = npad
    else:
        npad = 1 << (nint - 1).bit_length()
        if F + npad > bits:
            npad = nint
        # blocks z, x': |z|'s planes from z, the mirror's sign from x' at the ring's msb
        zs = _wsum(sess, None, (), x=xt, wx=1, cblk=(0,), second=(C, 0), lead=True)
        if zs is None:
            z = rep.lincomb(sess, [(C, xt)])
            zs = concat(sess, [RepFixed(z, F, integ), RepFixed(xt, fx, integ)], 0).t
        bd = rep.bit_decompose(sess, zs)
        ab = rep.b2a_planes_xor(sess, bd, F - f, f + npad, q, bits, blocks=2,
                                sbit=bits - 1)  # f + npad planes, then s
        rows = local(sess, ab, "Slice", slice=(0, f + npad, None))
        s = local(sess, ab, "IndexAxis", axis=0, index=f + npad)
        cs, nint_used = None, nint
    merged = (getattr(sess, "party_dot_trunc", None) is not None
              and hasattr(sess, "p_cross_plain") and npad >= 2 and npad & (npad - 1) == 0)
    e = _exp2_from_planes(sess, rows, f, integ, bits, nint_used, npad, True, merged, cs=cs,
                          plus=plus)
    return s, e

def softmax(sess, x: RepFixed, axis: int, upmost_index: int) -> RepFixed:
    """Reference softmax.rs:55-70: the comparison tree is unrolled over ``upmost_index``
    slices of ``axis`` (the axis length when the shape is static), so it lowers without
    concrete shapes."""
    shape = static_shape(sess, x)
    n = upmost_index if shape is None else min(shape[axis], upmost_index)
    cols = [local(sess, x, "IndexAxis", axis=axis, index=i) for i in range(n)]
    mx = maximum(sess, cols)
    mxe = local(sess, mx, "ExpandDims", axis=[axis])
    shifted = _with(x, rep.sub(sess, x.t, _bcast(sess, mxe.t, x.t)))
    e = exp_nonpositive(sess, shifted)
    ssum = local(sess, e, "Sum", axis=axis)  # >= 1 (the max term is e^0)
    inv = reciprocal_positive(sess, ssum)
    inve = local(sess, inv, "ExpandDims", axis=[axis])
    return mul(sess, e, _with(inve, _bcast(sess, inve.t, e.t)))


def _bcast(sess, small: RepTensor, big: RepTensor) -> RepTensor:
    return broadcast_like(sess, small, big)


def argmax(sess, x: RepFixed, axis: int, upmost_index: int) -> RepTensor:
    """Index of the maximum along ``axis`` as an arithmetic Z_2^64 sharing: a tree of
    (value, index) pairs reduced with less + mux (reference argmax.rs:6-96).  Each tree
    level is ONE stacked comparison over all its pairs and ONE mux that selects values
    and indices together."""
    shape = static_shape(sess, x)
    n = upmost_index if shape is None else min(shape[axis], upmost_index)
    vals = [local(sess, x, "IndexAxis", axis=axis, index=i) for i in range(n)]
    bits = x.bits
    vshape = static_shape(sess, vals[0])

    def index_const(i):
        if vshape is not None:
            return rep.from_public(sess, x.plc, R.fill(vshape, i, bits, sess.device), bits)
        # shape-polymorphic: a public scalar broadcast to the slices' run-time shape
        c = rep.from_public(sess, x.plc, R.fill((), i, bits, sess.device), bits)
        return broadcast_like(sess, c, vals[0].t)

    idx = [RepFixed(index_const(i), 0, x.integ) for i in range(n)]
    pairs = list(zip(vals, idx))
    while len(pairs) > 1:
        h = len(pairs) // 2
        va = _stack0(sess, [p[0] for p in pairs[0:2 * h:2]])
        vb = _stack0(sess, [p[0] for p in pairs[1:2 * h:2]])
        ia = _stack0(sess, [p[1] for p in pairs[0:2 * h:2]])
        ib = _stack0(sess, [p[1] for p in pairs[1:2 * h:2]])
        lt = rep.less_than_zero_arith(sess, rep.sub(sess, va.t, vb.t))  # a < b
        lt2 = concat(sess, [lt, lt], 0)
        sel = rep.mux(sess, lt2, concat(sess, [vb, ib], 0).t, concat(sess, [va, ia], 0).t)
        both = _unstack0(sess, _with(va, sel), 2 * h)
        nxt = [(both[i], RepFixed(both[h + i].t, 0, x.integ)) for i in range(h)]
        if len(pairs) % 2:
            nxt.append(pairs[-1])
        pairs = nxt
    out = pairs[0][1].t
    return rep.ring_cast(sess, out, 64) if bits != 64 else out
