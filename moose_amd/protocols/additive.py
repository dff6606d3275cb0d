"""Two-party additive secret sharing (the reference's ``additive`` dialect).

Parity: reference ``moose/src/additive`` -- ``AdtTensor{shares:[T;2]}`` on an
``AdditivePlacement{owners:[Role;2]}`` (``additive/mod.rs:19-50``), local linear ops
(``ops.rs``), ``RepToAdt`` (``convert.rs:12-80``), dealer-generated DaBits
(``dabit.rs:38-69``) and probabilistic truncation with a dealer mask
(``trunc.rs:35-62, 114-170``).  In this framework the additive dialect is the
intermediate form of the replicated TruncPr (rep -> adt -> truncate -> rep), and is
usable on its own through these functions.

Correlated randomness: the dealer shares one PRF key with each owner (for the
replicated use these are the rep setup keys k_0 [P0,P2] and k_2 [P1,P2]), so masks that
one owner can re-derive are never sent -- only the second owner's correction terms
travel (the reference ships full tensors, TODO at ``trunc.rs:51-52``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

from moose_amd.ir.computation import AdditivePlacement
from moose_amd.runtime.session import HV


@dataclass
class AdtTensor:
    plc: AdditivePlacement
    bits: int
    s0: HV  # share of owners[0]
    s1: HV  # share of owners[1]


def share(sess, plc: AdditivePlacement, x: HV, key: bytes = None, nonce: int = None) -> AdtTensor:
    """Owner x.host splits x = r + (x - r); r from a fresh seed sent to the other owner
    (a seed, not a tensor)."""
    bits = x.v.bits
    o0, o1 = plc.owners
    shape = sess.h("Shape", x.host, x)
    seed = sess.h_fresh_seed(x.host)
    r_here = sess.h("SampleSeeded", x.host, shape, seed, bits=bits)
    rest = sess.h("Sub", x.host, x, r_here)
    other = o1 if x.host == o0 else o0
    r_there = sess.h("SampleSeeded", other, sess.move(shape, other), sess.move(seed, other),
                     bits=bits)
    if x.host == o0:
        return AdtTensor(plc, bits, rest, r_there)
    if x.host == o1:
        return AdtTensor(plc, bits, r_there, rest)
    return AdtTensor(plc, bits, sess.move(rest, o0), r_there)


def reveal(sess, x: AdtTensor, host: str) -> HV:
    return sess.h("Add", host, x.s0, x.s1)


def add(sess, x: AdtTensor, y: AdtTensor) -> AdtTensor:
    o0, o1 = x.plc.owners
    return AdtTensor(x.plc, x.bits, sess.h("Add", o0, x.s0, y.s0), sess.h("Add", o1, x.s1, y.s1))


def sub(sess, x: AdtTensor, y: AdtTensor) -> AdtTensor:
    o0, o1 = x.plc.owners
    return AdtTensor(x.plc, x.bits, sess.h("Sub", o0, x.s0, y.s0), sess.h("Sub", o1, x.s1, y.s1))


def neg(sess, x: AdtTensor) -> AdtTensor:
    o0, o1 = x.plc.owners
    return AdtTensor(x.plc, x.bits, sess.h("Neg", o0, x.s0), sess.h("Neg", o1, x.s1))


def add_public(sess, x: AdtTensor, c) -> AdtTensor:
    """x + c with public c (added by the first owner only)."""
    o0, _ = x.plc.owners
    return AdtTensor(x.plc, x.bits, sess.h("Add", o0, x.s0, c), x.s1)


def mul_public(sess, x: AdtTensor, c) -> AdtTensor:
    o0, o1 = x.plc.owners
    return AdtTensor(x.plc, x.bits, sess.h("Mul", o0, x.s0, c), sess.h("Mul", o1, x.s1, c))


def shl(sess, x: AdtTensor, k: int) -> AdtTensor:
    o0, o1 = x.plc.owners
    return AdtTensor(x.plc, x.bits, sess.h("Shl", o0, x.s0, amount=k),
                     sess.h("Shl", o1, x.s1, amount=k))


# ---------------------------------------------------------------------------
# conversions with the replicated dialect
# ---------------------------------------------------------------------------
def from_rep(sess, x, plc: AdditivePlacement = None) -> AdtTensor:
    """RepToAdt without communication: with owners (P_i, P_j) of the replicated
    placement, P_i keeps x_i + x_{i+1} and P_j the remaining slot (which it holds)."""
    rp = x.plc
    o = rp.owners
    plc = plc or AdditivePlacement((o[0], o[1]))
    i, j = o.index(plc.owners[0]), o.index(plc.owners[1])
    a = sess.h("Add", o[i], sess.take(x.s0, i), sess.take(x.s1, i))
    k = (i + 2) % 3  # the slot P_i does not hold
    b = sess.take(x.s0, j) if j == k else sess.take(x.s1, j)
    return AdtTensor(plc, x.bits, a, b)


def to_rep(sess, rep_plc, y: AdtTensor, nonces: Tuple[int, int] = None, shapes=None):
    """AdtToRep for owners (P0, P1) of ``rep_plc`` (reference convert.rs:392-497):
    z0 = PRF(k_0) [P0, P2], z2 = PRF(k_2) [P1, P2], z1 = (y0 - z0) + (y1 - z2)
    exchanged between P0 and P1 -- one round, no dealer message."""
    from moose_amd.protocols.replicated import RepTensor

    p0, p1, p2 = rep_plc.owners
    if tuple(y.plc.owners) != (p0, p1):
        raise ValueError("adt -> rep expects the additive owners to be the first two parties")
    bits = y.bits
    if shapes is None:
        sh = [sess.h("Shape", h, v) for h, v in ((p0, y.s0), (p1, y.s1))]
        sh.append(sess.move(sh[0], p2))
    else:
        sh = list(shapes)
    n0, n2 = nonces if nonces is not None else (sess.nonce(rep_plc), sess.nonce(rep_plc))
    z0_at0 = sess.h_prf(rep_plc, p0, 0, sh[0], bits, n0)
    z2_at1 = sess.h_prf(rep_plc, p1, 2, sh[1], bits, n2)
    z0_at2 = sess.h_prf(rep_plc, p2, 0, sh[2], bits, n0)
    z2_at2 = sess.h_prf(rep_plc, p2, 2, sh[2], bits, n2)
    w0 = sess.h("Sub", p0, y.s0, z0_at0)
    w1 = sess.h("Sub", p1, y.s1, z2_at1)
    z1_at0 = sess.h("Add", p0, w0, sess.move(w1, p0))
    z1_at1 = sess.h("Add", p1, w1, sess.move(w0, p1))
    s0 = sess.gather(rep_plc, [z0_at0, z1_at1, z2_at2])
    s1 = sess.gather(rep_plc, [z1_at0, z2_at1, z0_at2])
    return RepTensor(rep_plc, bits, "arith", s0, s1)


# ---------------------------------------------------------------------------
# dealer-assisted protocols
# ---------------------------------------------------------------------------
def dabit(sess, rep_plc, shape: HV, bits: int, nonces: Tuple[int, int, int]):
    """A random bit b known to nobody but the dealer P2, additively shared between P0
    and P1 both in Z_2^bits and in Z_2 (reference dabit.rs:38-69).  P0's shares are
    PRF(k_0) draws; only P1's corrections are sent."""
    p0, p1, p2 = rep_plc.owners
    plc = AdditivePlacement((p0, p1))
    nb, na, nx = nonces
    sh2 = sess.move(shape, p2)
    sh0 = sess.move(shape, p0)
    b = sess.h("BitExtract", p2, sess.h_prf(rep_plc, p2, 2, sh2, 64, nb), bit_idx=0)
    b_ring = sess.h("RingInject", p2, b, bit_idx=0, bits=bits)
    a0_at2 = sess.h_prf(rep_plc, p2, 0, sh2, bits, na)
    x0_at2 = sess.h("BitExtract", p2, sess.h_prf(rep_plc, p2, 0, sh2, 64, nx), bit_idx=0)
    a1 = sess.move(sess.h("Sub", p2, b_ring, a0_at2), p1)
    x1 = sess.move(sess.h("Xor", p2, b, x0_at2), p1)
    a0 = sess.h_prf(rep_plc, p0, 0, sh0, bits, na)
    x0 = sess.h("BitExtract", p0, sess.h_prf(rep_plc, p0, 0, sh0, 64, nx), bit_idx=0)
    return AdtTensor(plc, bits, a0, a1), AdtTensor(plc, 1, x0, x1)


def trunc_pr(sess, rep_plc, x: AdtTensor, m: int, nonces, shapes=None) -> AdtTensor:
    """Probabilistic truncation of an additive sharing over Z_2^k by ``m`` bits with
    dealer P2 (Escudero et al., reference trunc.rs:114-170).  Valid for |x| < 2^(k-2);
    the result is off by at most one unit in the last place.

    r = r0 + r1 with r0 = PRF(k_0) [P0, P2] and r1 = PRF(k_2) [P1, P2] needs no message;
    the dealer sends P1 its shares of r_top and r_msb (P0 re-derives its own); P0 and P1
    then open c = x + r + 2^(k-2) to each other (one round)."""
    p0, p1, p2 = rep_plc.owners
    bits = x.bits
    k = bits - 1
    nr0, nr1, nt, nm = nonces
    if shapes is None:
        sh0 = sess.h("Shape", p0, x.s0)
        sh1 = sess.h("Shape", p1, x.s1)
        sh2 = sess.move(sh0, p2)
    else:  # every party already knows the shape (e.g. from its replicated shares)
        sh0, sh1, sh2 = shapes
    r = sess.h("Add", p2, sess.h_prf(rep_plc, p2, 0, sh2, bits, nr0),
               sess.h_prf(rep_plc, p2, 2, sh2, bits, nr1))
    r_msb = sess.h("Shr", p2, r, amount=bits - 1)
    r_top = sess.h("Shr", p2, sess.h("Shl", p2, r, amount=1), amount=m + 1)
    rt1 = sess.move(sess.h("Sub", p2, r_top, sess.h_prf(rep_plc, p2, 0, sh2, bits, nt)), p1)
    rm1 = sess.move(sess.h("Sub", p2, r_msb, sess.h_prf(rep_plc, p2, 0, sh2, bits, nm)), p1)
    r0 = sess.h_prf(rep_plc, p0, 0, sh0, bits, nr0)
    rt0 = sess.h_prf(rep_plc, p0, 0, sh0, bits, nt)
    rm0 = sess.h_prf(rep_plc, p0, 0, sh0, bits, nm)
    r1 = sess.h_prf(rep_plc, p1, 2, sh1, bits, nr1)
    mk0 = sess.h("Add", p0, sess.h("AddConst", p0, x.s0, value=1 << (k - 1), bits=bits), r0)
    mk1 = sess.h("Add", p1, x.s1, r1)
    c_at0 = sess.h("Add", p0, mk0, sess.move(mk1, p0))
    c_at1 = sess.h("Add", p1, mk1, sess.move(mk0, p1))
    outs = []
    for host, c, rt, rm, first in ((p0, c_at0, rt0, rm0, True), (p1, c_at1, rt1, rm1, False)):
        c_msb = sess.h("Shr", host, c, amount=bits - 1)
        # share of the overflow bit r_msb XOR c_msb = rm + [first] c_msb - 2 c_msb rm
        ov = sess.h("Sub", host, rm, sess.h("Shl", host, sess.h("Mul", host, c_msb, rm), amount=1))
        if first:
            ov = sess.h("Add", host, ov, c_msb)
        y = sess.h("Sub", host, sess.h("Shl", host, ov, amount=k - m), rt)
        if first:
            c_top = sess.h("Shr", host, sess.h("Shl", host, c, amount=1), amount=m + 1)
            y = sess.h("Add", host, y, c_top)
            y = sess.h("AddConst", host, y, value=-(1 << (k - 1 - m)), bits=bits)
        outs.append(y)
    return AdtTensor(x.plc, bits, outs[0], outs[1])
