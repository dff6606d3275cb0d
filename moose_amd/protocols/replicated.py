"""Three-party replicated secret sharing (RSS) over Z_2^64, Z_2^128 and Z_2.

A secret x = x_0 + x_1 + x_2 (XOR for boolean sharings) is held as ``slots``: party p
holds (x_p, x_{p+1}).  A :class:`RepTensor` keeps the two party vectors ``s0`` (x_p at
party p) and ``s1`` (x_{p+1} at party p); ``s1`` is ``s0`` shifted by one party.

Correlated randomness: party p holds PRF keys k_p and k_{p+1} (so slot s can be sampled
by exactly the two parties holding slot s) and one key k_all common to all three (kept in
the setup; input sharing no longer draws from it: its third slot is zero, as the
reference's).

Parity with the reference (``moose/src/replicated``):

=====================  =====================================  =========================
protocol               reference                              rounds here
=====================  =====================================  =========================
share (owner member)   convert.rs:74-125                      1 msg (x_{j+1} -> P_{j+1})
share (outsider)       convert.rs:126-156                     1 (x sent + seeds)
reveal                 convert.rs:280-313                     1
add/sub/neg/sum/shape  arith.rs:7-314, ops.rs                 0
mul                    arith.rs:317-367                       1 (fused kernel + roll)
dot                    arith.rs:436-492                       1 (one K-doubled GEMM)
trunc_pr               fixedpoint.rs:80-103, additive/trunc   2 (dealer msgs overlap)
bit_decompose          bits.rs:6-21, misc.rs:181-243          1 + 1 + log2(k)
msb / less / greater   arith.rs:611-653, compare.rs           bit_decompose + 2
b2a (ring_inject)      convert.rs:316-390                     2
equal_zero / equal     compare.rs:24-89                       bit_decompose + log2(k)
mux                    control_flow.rs:9-45                   1 (+2 for a bit selector)
=====================  =====================================  =========================

Boolean sharings of k-bit words keep the k bits packed in one ring word (a Z_2^64 /
Z_2^128 element), so a Kogge-Stone level is ONE boolean multiplication of whole words
instead of k bit tensors (reference bits.rs stacks a [k, ...] bit array).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch

from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ops import ring as R
from moose_amd.runtime.session import HV
from moose_amd.runtime.session import PV
from moose_amd.runtime.session import Public
from moose_amd.utils.telemetry import span


@dataclass
class RepTensor:
    plc: ReplicatedPlacement
    bits: int  # 1, 64 or 128
    kind: str  # "arith" (additive) or "bool" (xor)
    s0: PV
    s1: PV
    # slot known to be zero by construction (a fresh input sharing sets slot j+2 = 0, as
    # the reference's; public knowledge of every party), else None
    zero_slot: Optional[int] = None

    @property
    def add_prim(self):
        return "Add" if self.kind == "arith" else "Xor"


class RawBits(RepTensor):
    """A boolean sharing of packed words held, for one party of a per-party session, as the
    Kogge-Stone adder's raw state ``raw`` = (p0, p1, g0, g1, t0, t1) (parallel/spmd.py
    p_bit_decompose): the sum words p ^ ((g ^ t) << 1) are computed when first read, and the
    B2A of bit planes reads the raw state directly (no sum kernel)."""

    def __init__(self, plc, bits, s0, s1, raw):
        self.raw = raw
        super().__init__(plc, bits, "bool", s0, s1)

    def _sum(self):
        if self._s0 is None:
            p0, p1, g0, g1, t0, t1 = self.raw
            zero0 = t0 if t0 is not None else R.zeros(g0.shape, g0.bits, g0.device)
            zero1 = t1 if t1 is not None else R.zeros(g1.shape, g1.bits, g1.device)
            o0, o1 = R.ks_sum2(p0, p1, g0, g1, zero0, zero1)
            self._s0, self._s1 = PV(self.plc, o0), PV(self.plc, o1)

    @property
    def s0(self):
        self._sum()
        return self._s0

    @s0.setter
    def s0(self, v):
        self._s0 = v

    @property
    def s1(self):
        self._sum()
        return self._s1

    @s1.setter
    def s1(self, v):
        self._s1 = v


class DeferredRep(RepTensor):
    """A product whose last reshare round has not run (parallel/party.py ``RoundB``): the
    shares are completed when first read, and a reveal to the dealer P2 merges that round
    with the reveal (session ``p_reveal_deferred``)."""

    def __init__(self, plc, bits, kind, s0, s1, tail):
        self._tail = tail
        super().__init__(plc, bits, kind, s0, s1)

    @property
    def s0(self):
        self._tail.finish()
        return self._s0

    @s0.setter
    def s0(self, v):
        self._s0 = v

    @property
    def s1(self):
        self._tail.finish()
        return self._s1

    @s1.setter
    def s1(self, v):
        self._s1 = v


# 2^m c of a public addend (a model bias): kept per (constant object, m) -- the constant's
# encoding is the same object every evaluation (ring.encode_lazy), so an evaluation adds
# it with one launch instead of a fill, a multiply and the add.  The entry holds the
# constant itself, so its id cannot be reused while cached.
_SCALED = {}


def _scaled_public(cv, m: int, bits: int):
    key = (id(cv), m, bits)
    hit = _SCALED.get(key)
    if hit is not None and hit[0] is cv:
        return hit[1]
    scaled = R.binary("mul", cv, R.fill((), 1 << m, bits, cv.data.device))
    capturing = cv.data.is_cuda and torch.cuda.is_current_stream_capturing()
    if len(_SCALED) < 1024 and not capturing and R.CONST_CACHE:
        _SCALED.setdefault(key, (cv, scaled))
    return scaled


class PendingTrunc(RepTensor):
    """A fixed-point product still 2^m above its type, held as this party's 3-out-of-3
    additive share ``v_add`` (a per-party dot before its tail:
    fixedpoint._dot_public_trunc_jobs), plus public addends at the truncated scale
    (``pubs``, party 0 adds them).  Reading the shares completes it with the batched tail
    (zero share + reshare + TruncPr by m: the dot's 2 rounds, as before).  The sigmoid's one
    bit decomposition takes the reshared untruncated value (:meth:`reshare_untruncated`, 1
    round -- it stays secret-shared); a reveal runs the dot tail and merges its round B with
    the reveal (:func:`_reveal_pending`, 2 rounds): no receiver ever holds shares of the
    untruncated value."""

    def __init__(self, sess, plc, bits, v_add, m, pubs=()):
        self._sess, self.v_add, self.m, self.pubs = sess, v_add, m, list(pubs)
        self.completed = False
        self._rb = None  # round B of a tail a reveal ran (shares pending until read)
        super().__init__(plc, bits, "arith", None, None)

    def with_public(self, c):
        return PendingTrunc(self._sess, self.plc, self.bits, self.v_add, self.m,
                            self.pubs + [c])

    def additive(self):
        """This party's additive share of 2^m (x + pubs) (members only)."""
        v = self.v_add
        if self._sess.party_index(self.plc) == 0 and self.pubs:
            for c in self.pubs:
                v = R.binary("add", v, _scaled_public(c.v if isinstance(c, Public) else c,
                                                      self.m, self.bits))
        return v

    def _complete(self):
        if self.completed:
            if self._rb is not None:
                self._rb.finish()
            return
        self.completed = True
        sess, plc, bits = self._sess, self.plc, self.bits
        nonces = tuple(sess.nonce(plc) for _ in range(7))
        member = sess.party_index(plc) is not None
        v = self.additive() if member else self.v_add
        like = PV(plc, v)
        r = tail_job(sess, plc, bits, self.m, nonces, like,
                     lambda o0, o1: R.MulJob(1, o0, o1, a=v.data.contiguous()))
        self._s0, self._s1 = r.s0, r.s1

    def reshare_untruncated(self):
        """Replicated shares of 2^m (x + pubs): zero share + one reshare round."""
        sess, plc = self._sess, self.plc
        member = sess.party_index(plc) is not None
        z = sess.p_add_zero_share(plc, PV(plc, self.additive() if member else self.v_add))
        return _reshare(sess, plc, z, self.bits, "arith")

    @property
    def s0(self):
        self._complete()
        return self._s0

    @s0.setter
    def s0(self, v):
        self._s0 = v

    @property
    def s1(self):
        self._complete()
        return self._s1

    @s1.setter
    def s1(self, v):
        self._s1 = v


def lazy(x) -> bool:
    """A replicated value with message rounds still pending (read-completed)."""
    return ((isinstance(x, PendingTrunc) and (not x.completed or x._rb is not None))
            or isinstance(x, DeferredRep))


def settle(x):
    """Run a lazy replicated value's pending rounds now (:func:`lazy`).  Lockstep groups
    (parallel/lockstep.py) settle the lazy inputs their units share before the coroutines
    start: a completion is not re-entrant, so two coroutines must not both run it."""
    if isinstance(x, PendingTrunc):
        x._complete()
    elif isinstance(x, DeferredRep):
        x._tail.finish()


def _reveal_pending(sess, x: PendingTrunc, host):
    """Open a PendingTrunc to a member P_j: the dot tail (zero share + reshare + TruncPr by
    m, round A) and then its round B merged with the reveal (parallel/party.py
    RoundB.reveal_to_member) -- 2 rounds instead of the tail's two plus the reveal, and the
    receiver sums shares of the TRUNCATED value only (reference: replicated/convert.rs:
    280-313 reveals the TruncPr'd tensor of replicated/fixedpoint.rs:80-103).  The shares
    stay pending until something reads them (round B then runs as usual).  None: the
    generic reveal."""
    from moose_amd.parallel.spmd import Remote

    plc = x.plc
    if host not in plc.owners or getattr(sess, "party_dot_trunc", None) is None \
            or not hasattr(sess, "party_exchange") or getattr(sess, "is_simulated", True):
        return None
    j = plc.owners.index(host)
    idx = sess.party_index(plc)
    nonces = tuple(sess.nonce(plc) for _ in range(7))  # as _complete: members and others
    x.completed = True
    if idx is None:
        r = PV(plc, Remote(x.bits))
        x._s0, x._s1 = r, r
        return HV(host, Remote(x.bits))
    v = x.additive()
    s0, s1, rb = sess.party_dot_trunc(plc, PV(plc, R.RT(v.data.contiguous().unsqueeze(0),
                                                        x.bits)), x.m, nonces, defer=True)
    x._s0 = PV(plc, R.RT(s0.v.data[0], x.bits))
    x._s1 = PV(plc, R.RT(s1.v.data[0], x.bits))
    x._rb = rb
    parts = rb.reveal_to_member(j)[0]
    if idx != j:
        return HV(host, Remote(x.bits))
    shape = v.data.shape
    return HV(host, R.opened(*[R.RT(t.reshape(shape), x.bits) for t in parts]))


def payload_bytes_of(v):
    return v.data.numel() * v.data.element_size()


def _owner_index(plc, host):
    try:
        return plc.owners.index(host)
    except ValueError:
        return None


# ---------------------------------------------------------------------------
# input / output
# ---------------------------------------------------------------------------
def share(sess, plc, x: HV, kind="arith") -> RepTensor:
    """Secret-share a ring tensor held by one host."""
    bits = x.v.bits if hasattr(x.v, "bits") else None
    with span("rep.share"):
        sess.setup(plc)
        shape = sess.h("Shape", x.host, x)
        j = _owner_index(plc, x.host)
        if j is None:
            return _share_outsider(sess, plc, x, kind, bits, shape)
        sub = "Sub" if kind == "arith" else "Xor"
        o = plc.owners
        j1, j2 = (j + 1) % 3, (j + 2) % 3
        n1, na = sess.nonce(plc), sess.nonce(plc)
        if getattr(sess, "fused", False):
            s0, s1 = sess.fused_share(plc, x, j, kind, n1, na)
            return RepTensor(plc, bits, kind, s0, s1, zero_slot=j2)
        party = getattr(sess, "party_share", None)
        if party is not None and bits in (64, 128):
            s0, s1 = party(plc, x, j, kind, n1, na)
            return RepTensor(plc, bits, kind, s0, s1, zero_slot=j2)
        d = sess.share_dir(plc, j) if hasattr(sess, "share_dir") else 1
        zero = lambda h: sess.h("Fill", o[h], shape, value=0, bits=bits)  # noqa: E731
        if d == 1:
            # as the reference (replicated/convert.rs:74-90): slot_j = PRF(k_j) [P_j,
            # P_{j+2}], slot_{j+1} = x - slot_j [P_j, sent to P_{j+1}], slot_{j+2} = 0.
            # Each single party other than the owner still misses one random slot
            r_j = sess.h_prf(plc, o[j], j, shape, bits, n1)
            r_j2 = sess.h_prf(plc, o[j2], j, shape, bits, n1)
            xj1 = sess.h(sub, o[j], x, r_j)
            comp0 = {j: r_j, j1: sess.move(xj1, o[j1]), j2: zero(j2)}
            comp1 = {j: xj1, j1: zero(j1), j2: r_j2}
        else:  # mirrored: slot_{j+1} = PRF(k_{j+1}) [P_j, P_{j+1}], slot_j -> P_{j+2}
            r_j = sess.h_prf(plc, o[j], j1, shape, bits, n1)
            r_j1 = sess.h_prf(plc, o[j1], j1, shape, bits, n1)
            xj = sess.h(sub, o[j], x, r_j)
            comp0 = {j: xj, j1: r_j1, j2: zero(j2)}
            comp1 = {j: r_j, j1: zero(j1), j2: sess.move(xj, o[j2])}
        s0 = sess.gather(plc, [comp0[i] for i in range(3)])
        s1 = sess.gather(plc, [comp1[i] for i in range(3)])
        return RepTensor(plc, bits, kind, s0, s1, zero_slot=j2)


def _share_outsider(sess, plc, x, kind, bits, shape):
    """Owner outside the placement: two fresh seeds go to the slot holders, the third
    slot x - PRG(seed0) - PRG(seed1) is sent to its two holders."""
    o = plc.owners
    sub = "Sub" if kind == "arith" else "Xor"
    seed0, seed1 = sess.h_fresh_seed(x.host), sess.h_fresh_seed(x.host)
    r0 = sess.h("SampleSeeded", x.host, shape, seed0, bits=bits)
    r1 = sess.h("SampleSeeded", x.host, shape, seed1, bits=bits)
    x2 = sess.h(sub, x.host, sess.h(sub, x.host, x, r0), r1)

    def expand(seed, host):
        return sess.h("SampleSeeded", host, sess.move(shape, host), sess.move(seed, host),
                      bits=bits)

    # slot0 = PRG(seed0) at P0, P2 ; slot1 = PRG(seed1) at P0, P1 ; slot2 = x2 at P1, P2
    s0 = sess.gather(plc, [expand(seed0, o[0]), expand(seed1, o[1]), sess.move(x2, o[2])])
    s1 = sess.gather(plc, [expand(seed1, o[0]), sess.move(x2, o[1]), expand(seed0, o[2])])
    return RepTensor(plc, bits, kind, s0, s1)


def reveal(sess, x: RepTensor, host: str) -> HV:
    """Open x to ``host`` (a party of x.plc or an outsider)."""
    with span("rep.reveal"):
        if isinstance(x, PendingTrunc) and not x.completed:
            r = _reveal_pending(sess, x, host)
            if r is not None:
                return r
        tail = getattr(x, "_tail", None)
        if tail is not None and not tail.done:
            fast = getattr(sess, "p_reveal_deferred", None)
            r = fast(x, tail, host) if fast is not None else None
            if r is not None:
                return r
        add = x.add_prim
        fast = getattr(sess, "p_reveal", None)
        if fast is not None and x.kind == "arith" and x.bits in (64, 128):
            r = fast(x, host)
            if r is not None:
                return r
        j = _owner_index(x.plc, host)
        if j is not None:
            # P_j holds (x_j, x_{j+1}); x_{j+2} comes from P_{j+1} (its s1)
            a = sess.h(add, host, sess.take(x.s0, j), sess.take(x.s1, j))
            c = sess.move(sess.take(x.s1, (j + 1) % 3), host)
            return sess.h(add, host, a, c)
        a = sess.move(sess.take(x.s0, 0), host)
        b = sess.move(sess.take(x.s1, 0), host)
        c = sess.move(sess.take(x.s1, 1), host)
        return sess.h(add, host, sess.h(add, host, a, b), c)


def from_public(sess, plc, value, bits, kind="arith") -> RepTensor:
    """Trivial sharing of a value every party knows: slots (v, 0, 0)."""
    s0 = sess.p_public_slot(plc, value, 0, bits)
    s1 = sess.p_public_slot(plc, value, 2, bits)
    return RepTensor(plc, bits, kind, s0, s1)


def from_slot_holders(sess, plc, slot: int, x_h0: HV, x_h1: HV, like: PV,
                      kind="arith") -> RepTensor:
    """Sharing of a value known to both holders of ``slot`` (party ``slot`` holds it as
    s0 -> ``x_h0``; party ``slot-1`` as s1 -> ``x_h1``): that slot = x, the others 0.
    No communication (e.g. x_2 of an arithmetic sharing in bit decomposition).  ``like``
    is any party vector of the same shape (each party takes its zeros' shape from it)."""
    bits = x_h0.v.bits if hasattr(x_h0.v, "bits") else None
    fused = getattr(sess, "p_from_slot_holders", None)
    if fused is not None:
        r = fused(plc, slot, x_h0, x_h1, like)
        if r is not None:
            return RepTensor(plc, bits, kind, r[0], r[1])
    o = plc.owners
    h0, h1 = slot, (slot - 1) % 3
    comps0, comps1 = [], []
    for p in range(3):
        zero = None
        if p != h0 or p != h1:
            shape = sess.h("Shape", o[p], sess.take(like, p))
            zero = sess.h("Fill", o[p], shape, value=0, bits=bits)
        comps0.append(x_h0 if p == h0 else zero)
        comps1.append(x_h1 if p == h1 else zero)
    return RepTensor(plc, bits, kind, sess.gather(plc, comps0), sess.gather(plc, comps1))


# ---------------------------------------------------------------------------
# local (communication-free) operations
# ---------------------------------------------------------------------------
def _sharewise(sess, prim, plc, a, b=None, **attrs):
    """prim on both share vectors: (prim(a[0], b[0]), prim(a[1], b[1])).  A stacked session
    does the pair in one kernel where it can (p_pair); otherwise two ops."""
    pair = getattr(sess, "p_pair", None)
    if pair is not None:
        r = pair(prim, plc, a, b, **attrs)
        if r is not None:
            return r
    if b is None:
        return sess.p(prim, plc, a[0], **attrs), sess.p(prim, plc, a[1], **attrs)
    return sess.p(prim, plc, a[0], b[0], **attrs), sess.p(prim, plc, a[1], b[1], **attrs)


def local(sess, x: RepTensor, prim, **attrs) -> RepTensor:
    """Apply a linear / shape primitive share-wise."""
    s0, s1 = _sharewise(sess, prim, x.plc, (x.s0, x.s1), **attrs)
    return RepTensor(x.plc, x.bits, x.kind, s0, s1)


def add(sess, x: RepTensor, y: RepTensor) -> RepTensor:
    s0, s1 = _sharewise(sess, x.add_prim, x.plc, (x.s0, x.s1), (y.s0, y.s1))
    return RepTensor(x.plc, x.bits, x.kind, s0, s1)


def sub(sess, x: RepTensor, y: RepTensor) -> RepTensor:
    a = "Sub" if x.kind == "arith" else "Xor"
    s0, s1 = _sharewise(sess, a, x.plc, (x.s0, x.s1), (y.s0, y.s1))
    return RepTensor(x.plc, x.bits, x.kind, s0, s1)


def neg(sess, x: RepTensor) -> RepTensor:
    if x.kind == "bool":
        return x
    return local(sess, x, "Neg")


def add_public(sess, x: RepTensor, c) -> RepTensor:
    """x + c for a public c (added to slot 0 only).  A PendingTrunc stays pending (the
    addend rides into its tail)."""
    if isinstance(x, PendingTrunc) and not x.completed:
        return x.with_public(c)
    return _apply_public(sess, x, x.add_prim, c)


def sub_public(sess, x: RepTensor, c) -> RepTensor:
    return _apply_public(sess, x, "Sub" if x.kind == "arith" else "Xor", c)


def _apply_public(sess, x: RepTensor, prim, c) -> RepTensor:
    """prim(share of party 0, c): slot 0 of s0 and slot 2 of s1 hold x_0."""
    both = getattr(sess, "p_apply_at2", None)
    if both is not None:
        r = both(prim, x.plc, x.s0, x.s1, 0, 2, c)
        if r is not None:
            return RepTensor(x.plc, x.bits, x.kind, r[0], r[1])
    s0 = sess.p_apply_at(prim, x.plc, x.s0, 0, c)
    s1 = sess.p_apply_at(prim, x.plc, x.s1, 2, c)
    return RepTensor(x.plc, x.bits, x.kind, s0, s1)


def public_sub(sess, c, x: RepTensor) -> RepTensor:
    return add_public(sess, neg(sess, x), c) if x.kind == "arith" else add_public(sess, x, c)


def mul_public(sess, x: RepTensor, c) -> RepTensor:
    m = "Mul" if x.kind == "arith" else "And"
    pc = sess.public(x.plc, c)
    s0, s1 = _sharewise(sess, m, x.plc, (x.s0, x.s1), (pc, pc))
    return RepTensor(x.plc, x.bits, x.kind, s0, s1)


def dot_public(sess, x: RepTensor, c, public_left=False) -> RepTensor:
    pc = sess.public(x.plc, c)
    pair = getattr(sess, "p_dot_public_pair", None)
    if pair is not None and not public_left:
        r = pair(x.plc, x.s0, x.s1, pc)
        if r is not None:
            return RepTensor(x.plc, x.bits, x.kind, r[0], r[1])
    if public_left:
        return RepTensor(x.plc, x.bits, x.kind, sess.p("Dot", x.plc, pc, x.s0),
                         sess.p("Dot", x.plc, pc, x.s1))
    return RepTensor(x.plc, x.bits, x.kind, sess.p("Dot", x.plc, x.s0, pc),
                     sess.p("Dot", x.plc, x.s1, pc))


def shl(sess, x: RepTensor, k: int) -> RepTensor:
    return local(sess, x, "Shl", amount=k)


def add_n(sess, xs) -> RepTensor:
    """sum of replicated values (one kernel for views of one stack on a stacked device
    session, else a chain of share-wise adds -- the same ring values)."""
    x = xs[0]
    f = getattr(sess, "p_add_n", None)
    if f is not None and x.kind == "arith" and len(xs) > 1:
        r = f(x.plc, [(t.s0, t.s1) for t in xs])
        if r is not None:
            return RepTensor(x.plc, x.bits, x.kind, r[0], r[1])
    acc = x
    for t in xs[1:]:
        acc = add(sess, acc, t)
    return acc


def lincomb(sess, terms, const=None) -> RepTensor:
    """sum_t k_t * x_t (+ public const) for arithmetic sharings of one shape and small integer
    k_t: one share-wise kernel on a stacked device session, else composed from neg / shl /
    mul_public / add (exactly the same ring values either way)."""
    x = terms[0][1]
    f = getattr(sess, "p_lincomb", None)
    if f is not None and x.kind == "arith":
        r = f(x.plc, [(k, t.s0, t.s1) for k, t in terms], const)
        if r is not None:
            return RepTensor(x.plc, x.bits, x.kind, r[0], r[1])

    def scaled(k, t):
        if k == 1:
            return t
        if k == -1:
            return neg(sess, t)
        if k in (2, -2):
            d = shl(sess, t, 1)
            return d if k == 2 else neg(sess, d)
        return mul_public(sess, t, R.fill((), int(k), t.bits, getattr(sess, "device", "cpu")))

    acc = scaled(*terms[0])
    for k, t in terms[1:]:
        acc = add(sess, acc, scaled(k, t))
    return acc if const is None else add_public(sess, acc, const)


def sum(sess, x: RepTensor, axis=None) -> RepTensor:  # noqa: A001
    return local(sess, x, "Sum", axis=axis)


# ---------------------------------------------------------------------------
# multiplication
# ---------------------------------------------------------------------------
def _reshare(sess, plc, z: PV, bits, kind) -> RepTensor:
    """z_p (already masked by a zero share) -> P_{p-1}: one communication round."""
    return RepTensor(plc, bits, kind, z, sess.shift(z, 1))


def mul(sess, x: RepTensor, y: RepTensor) -> RepTensor:
    """Elementwise product (AND for boolean sharings): one fused kernel + one round."""
    with span("rep.mul"):
        kind = x.kind
        fused = getattr(sess, "p_mul_reshare", None)
        if fused is not None and getattr(sess, "fused", False):
            s0, s1 = fused(kind, x.plc, x.s0, x.s1, y.s0, y.s1)
            return RepTensor(x.plc, x.bits, kind, s0, s1)
        z = sess.p_cross(kind, x.plc, x.s0, x.s1, y.s0, y.s1, zero_share=True)
        return _reshare(sess, x.plc, z, x.bits, kind)


def mul_public_trunc(sess, x: RepTensor, c, m: int, value: int = None) -> RepTensor:
    """trunc_pr(mul_public(x, c), m); for a public scalar ring constant whose integer
    ``value`` the caller knows, on a fused stacked session, the multiplication runs inside the
    TruncPr kernel (same shares); on a per-party session inside the batched tail."""
    if (m and 0 < m <= 63 and value is not None and -(1 << 62) < value < (1 << 62)
            and jobs_ok(sess, x)):
        return mul_public_trunc_jobs(sess, x, value, m)
    if (m and value is not None and x.kind == "arith" and getattr(sess, "fused", False)
            and x.bits in (64, 128) and hasattr(sess, "fused_trunc_pr_premul")):
        with span("rep.trunc_pr"):
            plc = x.plc
            nonces = tuple(sess.nonce(plc) for _ in range(6))  # as trunc_pr draws them
            s0, s1 = sess.fused_trunc_pr_premul(x, m, nonces, value)
            return RepTensor(plc, x.bits, "arith", s0, s1)
    return trunc_pr(sess, mul_public(sess, x, c), m)


def mul_trunc(sess, x: RepTensor, y: RepTensor, m: int, out=None) -> RepTensor:
    """trunc_pr(mul(x, y), m): one fused kernel on a stacked device session for small
    operands (same shares as the two steps), the two protocol steps otherwise."""
    f = getattr(sess, "p_mul_trunc", None)
    if f is not None and m and x.kind == "arith" and getattr(sess, "fused", False):
        r = f(x.plc, x.s0, x.s1, y.s0, y.s1, m, out=out)
        if r is not None:
            return RepTensor(x.plc, x.bits, "arith", r[0], r[1])
    jobs = getattr(sess, "party_jobs", None)
    if jobs is not None and sess.party_index(x.plc) is not None:
        one = [t for t in (x, y) if t.s0.v.numel() == 1]
        if len(one) == 1 and x.s0.v.shape != y.s0.v.shape:
            # a one-element factor (a learning rate, a momentum): broadcast inside the tail
            # kernel as a stride-0 row when the product goes there, else materialised
            r = _mul_trunc_bcast(sess, x, y, m, out)
            if r is not None:
                return r
            small = one[0]
            big = y if small is x else x
            b = local(sess, small, "Broadcast", shape=tuple(big.s0.v.shape))
            x, y = (b, y) if small is x else (x, b)
    if (jobs is not None and JOBS and 0 < m <= 63 and x.kind == "arith" and x.bits in (64, 128)
            and os.environ.get("MOOSEX_DOT_TAIL", "1") != "0" and sess.jobs_shape_ok(x, y)):
        # one party of a per-party session: the product's cross terms inside the batched
        # tail's first kernel (csrc/rss_jobs.hip) -- 3 kernels, bitwise the shares of the
        # cross-term kernel + dot tail below (same nonces, same element order)
        with span("rep.mul_trunc_party"):
            nonces = tuple(sess.nonce(x.plc) for _ in range(7))
            return _mul_trunc_jobs(sess, x, y, m, nonces, out)
    party = getattr(sess, "party_dot_trunc", None)
    plain = getattr(sess, "p_cross_plain", None)
    if (party is not None and plain is not None and 0 < m <= 63 and x.kind == "arith"
            and x.bits in (64, 128) and os.environ.get("MOOSEX_DOT_TAIL", "1") != "0"):
        # the dot's per-party tail (parallel/party.py) on the elementwise cross products:
        # the reshare folded into TruncPr's first round -- 2 rounds instead of 3, the same
        # nonces in the same order as the fused stacked kernel (same shares)
        with span("rep.mul_trunc_party"):
            nonces = tuple(sess.nonce(x.plc) for _ in range(7))
            v = plain("arith", x.plc, x.s0, x.s1, y.s0, y.s1)
            s0, s1 = party(x.plc, v, m, nonces, out=(out[0], out[1]) if out else None)
            return RepTensor(x.plc, x.bits, "arith", s0, s1)
    return trunc_pr(sess, mul(sess, x, y), m, out=out)


# per-party sessions batch products into the tail kernels of csrc/rss_jobs.hip
JOBS = os.environ.get("MOOSEX_PARTY_JOBS", "1") != "0"


def _mul_trunc_bcast(sess, x: RepTensor, y: RepTensor, m: int, out=None):
    """mul_trunc of a dense operand by a one-element one on a per-party session, through
    the batched tail with the small factor as a stride-0 row (rows of length 1): the same
    elements in the same order as the product of the materialised broadcast, so the same
    shares.  None when the tail cannot take it."""
    big, small = (x, y) if y.s0.v.numel() == 1 else (y, x)
    if not (JOBS and 0 < m <= 63 and x.kind == "arith" and y.kind == "arith"
            and x.bits in (64, 128) and os.environ.get("MOOSEX_DOT_TAIL", "1") != "0"):
        return None
    shares = [t.v for r in (big, small) for t in (r.s0, r.s1)]
    if not all(isinstance(t, R.RT) and t.data.is_contiguous() for t in shares):
        return None
    n = big.s0.v.numel()
    with span("rep.mul_trunc_party"):
        nonces = tuple(sess.nonce(x.plc) for _ in range(7))
        return tail_job(sess, x.plc, x.bits, m, nonces, big.s0,
                        lambda o0, o1: R.MulJob(n, o0, o1,
                                                x=(big.s0.v.data, big.s1.v.data), sx=1,
                                                y=(small.s0.v.data, small.s1.v.data), sy=0),
                        out=out, L=1)


def _mul_trunc_jobs(sess, x: RepTensor, y: RepTensor, m: int, nonces, out=None) -> RepTensor:
    return tail_job(sess, x.plc, x.bits, m, nonces, x.s0,
                    lambda o0, o1: R.MulJob(1, o0, o1, x=(x.s0.v.data, x.s1.v.data),
                                            y=(y.s0.v.data, y.s1.v.data)), out=out)


def tail_job(sess, plc, bits, m, nonces, like: PV, make, out=None, L=None) -> RepTensor:
    """One value through the per-party batched tail (csrc/rss_jobs.hip): ``make(o0, o1)``
    builds its ring.MulJob (one row of ``like``'s size, or rows of length ``L``) writing
    the new shares to o0 / o1.  Non-members get placeholders."""
    from moose_amd.parallel.spmd import Remote

    if sess.party_index(plc) is None:
        r = PV(plc, Remote(bits))
        return RepTensor(plc, bits, "arith", r, r)
    v = like.v
    if out is not None:
        o0, o1 = out[0].v.data, out[1].v.data
    else:
        o0, o1 = R.empty2(v.shape, bits, v.data.device)
        o0, o1 = o0.data, o1.data
    sess.party_jobs(plc, [make(o0, o1)], L if L is not None else max(1, v.numel()), bits, m,
                    nonces)
    return RepTensor(plc, bits, "arith", PV(plc, R.RT(o0, bits)), PV(plc, R.RT(o1, bits)))


def jobs_ok(sess, *reps) -> bool:
    """A per-party session whose products run through the batched tail kernels: every share
    of every operand one dense shape (members decide alike; non-members follow)."""
    if getattr(sess, "party_jobs", None) is None or not JOBS:
        return False
    if os.environ.get("MOOSEX_DOT_TAIL", "1") == "0" or reps[0].bits not in (64, 128):
        return False
    return all(r.kind == "arith" for r in reps) and sess.jobs_shape_ok(*reps)


def mul_public_trunc_jobs(sess, x: RepTensor, value: int, m: int) -> RepTensor:
    """trunc_pr(x * c, m) for a public integer c = ``value`` on a per-party session: the
    additive shares c x_p (each party's first share component scaled) through the batched
    tail -- 3 kernels, 2 rounds (the generic path multiplies both components first)."""
    with span("rep.trunc_pr"):
        nonces = tuple(sess.nonce(x.plc) for _ in range(7))
        return tail_job(sess, x.plc, x.bits, m, nonces, x.s0,
                        lambda o0, o1: R.MulJob(1, o0, o1, a=x.s0.v.data, ca=value))


def mul_trunc_many(sess, jobs):
    """Independent fixed-point products [(x, y, m, out)] of one placement: two of them in ONE
    launch on a stacked device session (p_mul_trunc2), else one by one -- the same nonces in
    the same order either way, so the same shares."""
    f = getattr(sess, "p_mul_trunc2", None)
    if (f is not None and len(jobs) == 2 and getattr(sess, "fused", False)
            and all(x.kind == "arith" and y.kind == "arith" and m for x, y, m, _ in jobs)):
        r = f(jobs[0][0].plc, [(x.s0, x.s1, y.s0, y.s1, m, out) for x, y, m, out in jobs])
        if r is not None:
            return [RepTensor(x.plc, x.bits, "arith", a, b)
                    for (x, _, _, _), (a, b) in zip(jobs, r)]
    return [mul_trunc(sess, x, y, m, out=out) for x, y, m, out in jobs]


def and_(sess, x: RepTensor, y: RepTensor) -> RepTensor:
    assert x.kind == "bool"
    return mul(sess, x, y)


def xor(sess, x: RepTensor, y: RepTensor) -> RepTensor:
    assert x.kind == "bool"
    return add(sess, x, y)


ZERO_SLOTS = os.environ.get("MOOSEX_ZERO_SLOTS", "0") == "1"


def _cross_terms(p, zx, zy):
    """The nonzero terms of party p's cross product x_p y_p + x_p y_{p+1} + x_{p+1} y_p
    given the operands' known-zero slots, as ONE product (a, b) of share expressions --
    a, b in {"x0", "x1", "x01", "y0", "y1", "y01"} (x0 = x_p, x1 = x_{p+1}, x01 = their
    sum) -- or None when all three terms are nonzero (two products needed)."""
    xp, xq = p != zx, (p + 1) % 3 != zx
    yp, yq = p != zy, (p + 1) % 3 != zy
    t1, t2, t3 = xp and yp, xp and yq, xq and yp
    if t1 and t2 and t3:
        return None
    if t1 and t2:
        return "x0", "y01"
    if t1 and t3:
        return "x01", "y0"
    if t1:
        return "x0", "y0"
    if t2:
        return "x0", "y1"
    if t3:
        return "x1", "y0"
    return "zero", "zero"


def _zero_slot_cross(sess, x: RepTensor, y: RepTensor):
    """The local cross products of a stacked-layout session ([3, M, K] party vectors) when
    the operands have known-zero slots (fresh input sharings): every party's product is a
    single K-long GEMM instead of the K-doubled one -- half the MFMA work, bitwise the same
    values.  Opt-in (MOOSEX_ZERO_SLOTS=1); None when it does not apply."""
    if not ZERO_SLOTS or x.zero_slot is None and y.zero_slot is None:
        return None
    xs0, xs1, ys0, ys1 = x.s0.v, x.s1.v, y.s0.v, y.s1.v
    if not all(isinstance(t, R.RT) for t in (xs0, xs1, ys0, ys1)):
        return None
    if len(xs0.shape) != 3 or len(ys0.shape) != 3 or x.bits not in (64, 128):
        return None
    terms = [_cross_terms(p, x.zero_slot, y.zero_slot) for p in range(3)]
    if any(t is None or t[0] == "zero" for t in terms):
        return None
    bits = x.bits

    def pick(name, s0, s1, p):
        a, b = R.RT(s0.data[p], bits), R.RT(s1.data[p], bits)
        return a if name[1:] == "0" else b if name[1:] == "1" else R.binary("add", a, b)

    A = torch.stack([pick(a, xs0, xs1, p).data for p, (a, _) in enumerate(terms)])
    B = torch.stack([pick(b, ys0, ys1, p).data for p, (_, b) in enumerate(terms)])
    return PV(x.plc, R.dot(R.RT(A, bits), R.RT(B, bits), nb=1))


def dot(sess, x: RepTensor, y: RepTensor, nbatch: int = 0) -> RepTensor:
    """Matrix product: z_p = x_p.(y_p + y_{p+1}) + x_{p+1}.y_p as ONE K-doubled MFMA
    GEMM (all parties batched when stacked), + zero share, + reshare.  ``nbatch``
    leading axes of x and y index independent products done in the same launches."""
    with span("rep.dot"):
        over = getattr(sess, "p_dot_zs_reshare", None)
        if over is not None and getattr(sess, "fused", False) and not nbatch:
            res = over(x.plc, x.s0, x.s1, y.s0, y.s1, x.kind)
            if res is not None:
                return RepTensor(x.plc, x.bits, x.kind, res[0], res[1])
        if nbatch:
            v = sess.p_dot_cross(x.plc, x.s0, x.s1, y.s0, y.s1, nbatch=nbatch)
        else:
            v = _zero_slot_cross(sess, x, y) or sess.p_dot_cross(x.plc, x.s0, x.s1, y.s0,
                                                                    y.s1)
        fused = getattr(sess, "p_zero_share_reshare", None)
        if fused is not None and getattr(sess, "fused", False):
            s0, s1 = fused(x.plc, v, x.kind)
            return RepTensor(x.plc, x.bits, x.kind, s0, s1)
        z = sess.p_add_zero_share(x.plc, v, x.kind)
        return _reshare(sess, x.plc, z, x.bits, x.kind)


def _rows(pv: PV, r0: int, r1: int) -> PV:
    """Rows [r0, r1) of a stacked party vector holding a 2-D tensor per party (a view)."""
    v = pv.v
    return PV(pv.plc, R.RT(v.data[:, r0:r1], v.bits))


def dot_trunc(sess, x: RepTensor, y: RepTensor, m: int, nbatch: int = 0) -> RepTensor:
    """trunc_pr(dot(x, y), m) -- the fixed-point matrix product.  ``nbatch`` leading axes of
    x and y index independent products (one batched GEMM, one tail).

    Sessions whose reshares cross GPUs set ``pipeline_chunks`` > 1: the product of 2-D
    operands then runs as a row-chunked pipeline.  The GEMM of row chunk c+1 runs on the
    main HIP stream while chunk c's zero share, reshare and TruncPr -- row-local, with all
    their RCCL exchanges -- run on the session's side stream, so the inter-GPU traffic of
    the dot hides behind the MFMA work (chunked RSS pipelines).  Every chunk is
    its own protocol instance (own nonces): a valid sharing of the same product, and two
    sessions that chunk alike produce bitwise-equal shares.  The y operand is limb-split
    once (p_prepare_cross) and x row blocks are read in place."""
    chunks = getattr(sess, "pipeline_chunks", 1)
    nchunk = 1
    if nbatch:
        if not (getattr(sess, "party_dot_trunc", None) is not None and m and 0 < m <= 63
                and x.kind == "arith" and x.bits in (64, 128)):
            return trunc_pr(sess, dot(sess, x, y, nbatch=nbatch), m)
        with span("rep.dot_trunc_party"):
            nonces = tuple(sess.nonce(x.plc) for _ in range(7))
            v = sess.p_dot_cross(x.plc, x.s0, x.s1, y.s0, y.s1, nbatch=nbatch)
            s0, s1 = sess.party_dot_trunc(x.plc, v, m, nonces)
            return RepTensor(x.plc, x.bits, "arith", s0, s1)
    if chunks > 1:
        xs, ys = x.s0.v.shape, y.s0.v.shape  # stacked: (3, M, K), (3, K, N)
        if len(xs) == 3 and len(ys) == 3:
            M = xs[1]
            nchunk = min(chunks, M // 128)
    party = getattr(sess, "party_dot_trunc", None)
    use_party = (party is not None and m and 0 < m <= 63 and x.kind == "arith"
                 and x.bits in (64, 128) and os.environ.get("MOOSEX_DOT_TAIL", "1") != "0")
    if nchunk <= 1:
        tail = getattr(sess, "p_zs_trunc", None)
        if (tail is not None and m and x.kind == "arith" and getattr(sess, "fused", False)
                and getattr(sess, "device", None) is not None and sess.device.type == "cuda"
                and os.environ.get("MOOSEX_DOT_TAIL", "1") != "0"):
            with span("rep.dot_trunc_fused"):
                v = _zero_slot_cross(sess, x, y) or sess.p_dot_cross(x.plc, x.s0, x.s1, y.s0,
                                                                        y.s1)
                s0, s1 = tail(x.plc, v, m)  # zero share + reshare + TruncPr: one kernel
                return RepTensor(x.plc, x.bits, "arith", s0, s1)
        if use_party:  # the per-party tail: reshare folded into TruncPr (2 rounds)
            with span("rep.dot_trunc_party"):
                nonces = tuple(sess.nonce(x.plc) for _ in range(7))  # as dot + trunc_pr
                # the dealer's messages first: they travel while the GEMM runs
                pre_fn = getattr(sess, "party_dot_trunc_pre", None)
                pre = pre_fn(x.plc, x, y, m, nonces) if pre_fn is not None else None
                v = _zero_slot_cross(sess, x, y) or sess.p_dot_cross(x.plc, x.s0, x.s1, y.s0,
                                                                        y.s1)
                if getattr(sess, "defer_reshare", False) and pre is not None:
                    # the last reshare round waits for the first reader (a reveal to the
                    # dealer merges it with the reveal)
                    s0, s1, rb = party(x.plc, v, m, nonces, pre=pre, defer=True)
                    return DeferredRep(x.plc, x.bits, "arith", s0, s1, rb)
                s0, s1 = (party(x.plc, v, m, nonces) if pre is None
                          else party(x.plc, v, m, nonces, pre=pre))
                return RepTensor(x.plc, x.bits, "arith", s0, s1)
        return trunc_pr(sess, dot(sess, x, y), m)
    with span("rep.dot_trunc_pipelined"):
        plc, bits, kind = x.plc, x.bits, x.kind
        bounds = [M * c // nchunk for c in range(nchunk + 1)]
        data = x.s0.v.data
        cuda = data.is_cuda
        main = torch.cuda.current_stream(data.device) if cuda else None
        side = sess.side_stream() if cuda else None
        prepared = sess.p_prepare_cross(plc, y.s0, y.s1)
        # every chunk's shares land in rows of the result (no concatenation afterwards)
        N = y.s0.v.shape[2]
        shp = (3, M, N) + ((2,) if bits == 128 else ())
        # a stacked device session: each chunk's whole tail is one kernel writing its rows of
        # the result's share-pair ring buffer
        rows_fused = (cuda and getattr(sess, "fused", False) and m and kind == "arith"
                      and bits in (64, 128) and getattr(sess, "p_zs_trunc_rows", None) is not None)
        if rows_fused:
            buf4 = torch.empty((4,) + shp[1:], dtype=data.dtype, device=data.device)
            out0, out1 = buf4[0:3], buf4[1:4]
        else:
            out0 = torch.empty(shp, dtype=data.dtype, device=data.device)
            out1 = torch.empty_like(out0)

        def tail(v, r0, r1):
            if rows_fused:
                sess.p_zs_trunc_rows(plc, v, m, buf4, r0)
                return
            if use_party:
                nonces = tuple(sess.nonce(plc) for _ in range(7))
                party(plc, v, m, nonces, out=(out0[:, r0:r1], out1[:, r0:r1]))
                return
            z = sess.p_add_zero_share(plc, v, kind)
            t = trunc_pr(sess, _reshare(sess, plc, z, bits, kind), m)
            out0[:, r0:r1].copy_(t.s0.v.data)
            out1[:, r0:r1].copy_(t.s1.v.data)

        for c in range(nchunk):
            r0, r1 = bounds[c], bounds[c + 1]
            v = sess.p_dot_cross_rows(plc, x.s0, x.s1, r0, r1, prepared)
            if not cuda:
                tail(v, r0, r1)
                continue
            ev = torch.cuda.Event()
            ev.record(main)
            with torch.cuda.stream(side):
                side.wait_event(ev)
                v.v.data.record_stream(side)
                tail(v, r0, r1)
        if cuda:
            main.wait_stream(side)
        return RepTensor(plc, bits, kind, PV(plc, R.RT(out0, bits)), PV(plc, R.RT(out1, bits)))


# ---------------------------------------------------------------------------
# probabilistic truncation (dealer-assisted, P2 = dealer)
# ---------------------------------------------------------------------------
def trunc_pr(sess, x: RepTensor, m: int, out=None) -> RepTensor:
    """y ~= x / 2^m (probabilistic rounding, error <= 1 ulp), for |x| < 2^(k-2).

    Escudero et al. (as in reference additive/trunc.rs:114-170) with dealer P2 and all
    masks derived from PRF keys instead of shipped tensors where possible:
      * r = r0 + r1 with r0 = PRF(k_0) [P0,P2] and r1 = PRF(k_2) [P1,P2]: no message;
      * shares of r_top, r_msb for P1 are the only dealer messages (input independent);
      * round 1: P0 and P1 exchange their masked shares -> both know c = x + r + 2^(k-2);
      * round 2: additive -> replicated exchange (w_0, w_1).

    ``out`` (fused stacked sessions only): (s0, s1) party-vector views written in place.
    """
    if m == 0:
        return x
    with span("rep.trunc_pr"):
        plc, bits = x.plc, x.bits
        nr0, nr1, nt, nm = (sess.nonce(plc) for _ in range(4))
        if getattr(sess, "fused", False):
            n0, n2 = sess.nonce(plc), sess.nonce(plc)
            if out is not None:
                s0, s1 = sess.fused_trunc_pr(x, m, (nr0, nr1, nt, nm, n0, n2), out=out)
            else:
                s0, s1 = sess.fused_trunc_pr(x, m, (nr0, nr1, nt, nm, n0, n2))
            return RepTensor(plc, bits, "arith", s0, s1)
        if out is not None:
            raise ValueError("trunc_pr(out=...) needs a fused stacked session")
        party = getattr(sess, "party_trunc", None)
        if party is not None and bits in (64, 128) and m <= 63:
            n0, n2 = sess.nonce(plc), sess.nonce(plc)
            s0, s1 = party(x, m, (nr0, nr1, nt, nm, n0, n2))
            return RepTensor(plc, bits, "arith", s0, s1)
        from moose_amd.protocols import additive

        # every party takes the shape from its own share: no metadata messages
        sh = [sess.h("Shape", plc.owners[i], sess.take(x.s0, i)) for i in range(3)]
        a = additive.from_rep(sess, x)  # P0: x0 + x1, P1: x2 (local)
        y = additive.trunc_pr(sess, plc, a, m, (nr0, nr1, nt, nm), shapes=sh)
        return additive.to_rep(sess, plc, y, shapes=sh)


# ---------------------------------------------------------------------------
# bit decomposition & comparisons (packed boolean words)
# ---------------------------------------------------------------------------
def bit_decompose(sess, x: RepTensor, width=None) -> RepTensor:
    """Arithmetic sharing of x in Z_2^k -> boolean sharing of its k bits packed in one
    word.  y = x_0 + x_1 is boolean-shared by P0, x_2 is a trivial boolean sharing
    (slot 2), and a packed Kogge-Stone adder computes y + x_2 (log2 k AND rounds).
    ``width``: only the low ``width`` bits are needed (the caller knows |x| < 2^(width-1)
    or reads no higher bit); a per-party session then runs ceil(log2(width - 1)) levels."""
    with span("rep.bit_decompose"):
        plc, bits = x.plc, x.bits
        whole = getattr(sess, "p_bit_decompose", None)
        r = None
        if whole is not None and x.kind == "arith":
            r = whole(plc, x) if width is None else whole(plc, x, width=width)
        if isinstance(r, RepTensor):  # a per-party session's raw adder state
            return r
        if r is not None:  # every step below in one kernel (same nonces, same shares)
            return RepTensor(plc, bits, "bool", r[0], r[1])
        o = plc.owners
        y = sess.h("Add", o[0], sess.take(x.s0, 0), sess.take(x.s1, 0))
        yb = share(sess, plc, y, kind="bool")
        x2 = from_slot_holders(sess, plc, 2, sess.take(x.s0, 2), sess.take(x.s1, 1), x.s0,
                               kind="bool")
        return binary_adder(sess, yb, x2)


def binary_adder(sess, a: RepTensor, b: RepTensor) -> RepTensor:
    """Packed-word Kogge-Stone: bits of a + b for boolean sharings a, b."""
    bits = a.bits
    p = xor(sess, a, b)
    g = and_(sess, a, b)
    pk = p
    d = 1
    fused = getattr(sess, "fused", False) or getattr(sess, "ks_fused", False)
    level = getattr(sess, "p_ks_level", None) if fused else None
    chain = getattr(sess, "p_ks_adder", None) if fused else None
    if chain is not None and bits in (64, 128):
        # stacked device session: the whole chain and the final p ^ (g << 1) in one kernel
        r = chain(a.plc, g.s0, g.s1, pk.s0, pk.s1, bits, sum_out=True)
        if r is not None:
            return RepTensor(a.plc, bits, "bool", r[0], r[1])
    party_chain = getattr(sess, "p_ks_chain", None) if fused else None
    if party_chain is not None and bits in (64, 128):
        # per-party session: each level's xor rides in the next level's kernel
        r = party_chain(a.plc, g.s0, g.s1, pk.s0, pk.s1, bits)
        if r is not None:
            return RepTensor(a.plc, bits, "bool", r[0], r[1])
    if level is not None and bits in (64, 128):
        # stacked session: each level (shifts, both ANDs, reshare, xor) is one kernel
        while d < bits:
            both = 2 * d < bits
            g0, g1, q0, q1 = level(a.plc, g.s0, g.s1, pk.s0, pk.s1, d, both)
            g = RepTensor(a.plc, bits, "bool", g0, g1)
            if both:
                pk = RepTensor(a.plc, bits, "bool", q0, q1)
            d *= 2
        return xor(sess, p, shl(sess, g, 1))
    while d < bits:
        # batch the two independent ANDs of this level in one round
        gs = shl(sess, g, d)
        ps = shl(sess, pk, d)
        if 2 * d < bits:
            both = _stack2(sess, pk, pk)
            other = _stack2(sess, gs, ps)
            prod = and_(sess, both, other)
            t, pk_new = _unstack2(sess, prod)
            pk = pk_new
        else:
            t = and_(sess, pk, gs)
        g = xor(sess, g, t)
        d *= 2
    carry = shl(sess, g, 1)
    return xor(sess, p, carry)


def _stack2(sess, x: RepTensor, y: RepTensor) -> RepTensor:
    return RepTensor(x.plc, x.bits, x.kind, sess.p_stack2(x.s0, y.s0), sess.p_stack2(x.s1, y.s1))


def _unstack2(sess, x: RepTensor):
    a0, b0 = sess.p_unstack2(x.s0)
    a1, b1 = sess.p_unstack2(x.s1)
    return (RepTensor(x.plc, x.bits, x.kind, a0, a1), RepTensor(x.plc, x.bits, x.kind, b0, b1))


def bit_extract(sess, x: RepTensor, i: int) -> RepTensor:
    """Bit i of a packed boolean sharing -> boolean bit sharing (Z_2)."""
    assert x.kind == "bool"
    s0, s1 = _sharewise(sess, "BitExtract", x.plc, (x.s0, x.s1), bit_idx=i)
    return RepTensor(x.plc, 1, "bool", s0, s1)


def b2a(sess, b: RepTensor, ring_bits: int) -> RepTensor:
    """Boolean bit -> arithmetic bit in Z_2^ring_bits (2 rounds):
    b = a XOR b2 with a = b0 ^ b1 known to P0 and b2 known to P1, P2;
    [b] = [a] + [b2] - 2 [a][b2]."""
    with span("rep.b2a"):
        plc = b.plc
        o = plc.owners
        if b.bits != 1:
            raise TypeError("b2a expects a bit sharing")
        whole = getattr(sess, "p_b2a", None)
        r = whole(plc, b, ring_bits) if whole is not None else None
        if r is not None:  # every step below in one kernel (same nonces, same shares)
            return RepTensor(plc, ring_bits, "arith", r[0], r[1])
        prep = getattr(sess, "p_b2a_prep", None)
        r = prep(plc, b, ring_bits) if prep is not None else None
        if r is not None:  # the local steps below in one kernel (same values)
            a_ring, B0, B1 = r
            A = share(sess, plc, a_ring, kind="arith")
            B = RepTensor(plc, ring_bits, "arith", B0, B1)
        else:
            a_bit = sess.h("Xor", o[0], sess.take(b.s0, 0), sess.take(b.s1, 0))
            a_ring = sess.h("RingInject", o[0], a_bit, bit_idx=0, bits=ring_bits)
            A = share(sess, plc, a_ring, kind="arith")
            b2_h0 = sess.h("RingInject", o[2], sess.take(b.s0, 2), bit_idx=0, bits=ring_bits)
            b2_h1 = sess.h("RingInject", o[1], sess.take(b.s1, 1), bit_idx=0, bits=ring_bits)
            B = from_slot_holders(sess, plc, 2, b2_h0, b2_h1, b.s0, kind="arith")
        AB = mul(sess, A, B)
        return lincomb(sess, [(1, A), (1, B), (-2, AB)])


def b2a_planes(sess, b: RepTensor, start: int, count: int, ring_bits: int) -> RepTensor:
    """b2a of bit planes start..start+count-1 of a packed boolean sharing (a new leading
    logical axis): BitSplit + b2a, one kernel on a stacked device session (same shares)."""
    f = getattr(sess, "p_b2a_planes", None)
    r = f(b.plc, b, start, count, ring_bits) if f is not None else None
    if r is not None:
        return RepTensor(b.plc, ring_bits, "arith", r[0], r[1])
    planes = RepTensor(b.plc, 1, "bool", *_sharewise(sess, "BitSplit", b.plc, (b.s0, b.s1),
                                                     start=start, count=count))
    return b2a(sess, planes, ring_bits)


def b2a_planes_xor(sess, b: RepTensor, start: int, count: int, xbit: int,
                   ring_bits: int, blocks: int = 1, sbit: int = 0) -> RepTensor:
    """b2a of bit planes start..start+count-1 of a packed boolean sharing, each XORed with
    plane ``xbit``, followed by sign rows: count + tail rows on a new leading axis.  With
    xbit the sign of a two's-complement z, the rows are the planes of |z| (exactly: ~z = -z
    - 1 for z < 0, so off by one unit of bit 0) -- ONE decomposition serves planes and
    signs (the XOR is local on boolean shares).  ``b`` holds ``blocks`` blocks concatenated
    on axis 0 (decomposed together); the planes are block 0's, and the tail rows:

    * blocks 1: sign(z) (plane xbit); blocks 3 (z, z - T, z + T): [z >= T] (NOT sign(z - T)),
      [z < -T] (sign(z + T)), sign(z), all at plane xbit;
    * ``sbit`` > 0 (the ring's msb): blocks 2 (z, x): sign(x); blocks 4 (z, x - T', x + T',
      x): [x >= T'], [x < -T'], sign(x) -- signs of x at plane sbit, right for every
      representable x whatever magnitude bound z's planes assume.

    One round pair on a per-party session (parallel/spmd.py p_b2a_planes_xor, csrc/
    bits_party.h plane_of, same shares); Slice + BitSplit + Xor + Concat + b2a otherwise."""
    if (sbit > 0) != (blocks in (2, 4)):
        raise ValueError("b2a_planes_xor: blocks 2 / 4 take a sign plane sbit, 1 / 3 do not")
    f = getattr(sess, "p_b2a_planes_xor", None)
    code = blocks | (sbit << 8)
    r = f(b.plc, b, start, count, xbit, ring_bits, blocks=code) if f is not None else None
    if r is not None:
        return RepTensor(b.plc, ring_bits, "arith", r[0], r[1])
    if blocks > 1:
        n = sess.p_shape(b.s0)[0] // blocks
        parts = [_sharewise(sess, "Slice", b.plc, (b.s0, b.s1), slice=(k * n, (k + 1) * n, None))
                 for k in range(blocks)]
    else:
        parts = [(b.s0, b.s1)]
    planes = _sharewise(sess, "BitSplit", b.plc, parts[0], start=start, count=count)
    xsg = _sharewise(sess, "BitSplit", b.plc, parts[0], start=xbit, count=1)
    xored = _sharewise(sess, "Xor", b.plc, planes, xsg)
    sp = sbit if sbit > 0 else xbit
    sgns = [_sharewise(sess, "BitSplit", b.plc, p, start=sp, count=1) for p in parts]

    def not_(sg):
        nt = add_public(sess, RepTensor(b.plc, 1, "bool", *sg),
                        R.fill((), 1, 1, getattr(sess, "device", "cpu")))
        return (nt.s0, nt.s1)

    if blocks == 1:
        tail = [xsg]
    elif blocks == 3:  # NOT sign(z - T), sign(z + T), sign(z)
        tail = [not_(sgns[1]), sgns[2], xsg]
    elif blocks == 2:  # sign(x)
        tail = [sgns[1]]
    else:  # NOT sign(x - T'), sign(x + T'), sign(x)
        tail = [not_(sgns[1]), sgns[2], sgns[3]]
    both = [sess.p("Concat", b.plc, xored[i], *[g[i] for g in tail], axis=0) for i in range(2)]
    return b2a(sess, RepTensor(b.plc, 1, "bool", both[0], both[1]), ring_bits)


def msb(sess, x: RepTensor) -> RepTensor:
    """Boolean sharing of the sign bit."""
    bd = bit_decompose(sess, x)
    return bit_extract(sess, bd, x.bits - 1)


def less_than_zero_arith(sess, x: RepTensor, width=None) -> RepTensor:
    """Arithmetic 0/1 sharing of [x < 0]: b2a of the sign bit (one kernel for the whole of
    it on a stacked device session, same shares).  ``width``: |x| < 2^(width - 1) is known
    (a fixed-point type's bound), so the sign is bit width - 1 -- a per-party session's
    adder then spans only the low ``width`` bits (fewer rounds)."""
    f = getattr(sess, "p_sign_arith", None)
    r = None
    if f is not None and x.kind == "arith":
        r = f(x.plc, x) if width is None else f(x.plc, x, width=width)
    if r is not None:
        return RepTensor(x.plc, x.bits, "arith", r[0], r[1])
    return b2a(sess, msb(sess, x), x.bits)


def less(sess, x: RepTensor, y: RepTensor) -> RepTensor:
    """[x < y] as a boolean bit sharing (msb of x - y)."""
    return msb(sess, sub(sess, x, y))


def greater(sess, x: RepTensor, y: RepTensor) -> RepTensor:
    return msb(sess, sub(sess, y, x))


def equal_zero(sess, x: RepTensor) -> RepTensor:
    """[x == 0] as a boolean bit: AND-tree over the complemented packed bits."""
    bd = bit_decompose(sess, x)
    z = add_public(sess, bd, R.fill((), (1 << x.bits) - 1, x.bits, sess.device))  # NOT
    w = x.bits
    while w > 1:
        w //= 2
        z = and_(sess, z, local(sess, z, "Shr", amount=w))
    return bit_extract(sess, z, 0)


def equal(sess, x: RepTensor, y: RepTensor) -> RepTensor:
    return equal_zero(sess, sub(sess, x, y))


def mul_add(sess, a: RepTensor, b: RepTensor, c: RepTensor) -> RepTensor:
    """a * b + c.  On a per-party session the product's reshare round is deferred until the
    shares are read -- a reveal of the result absorbs it (one round fewer)."""
    f = getattr(sess, "p_mul_add_deferred", None)
    if f is not None:
        r = f(a.plc, a, b, c)
        if r is not None:
            return r
    return add(sess, mul(sess, a, b), c)


def mul_add_trunc(sess, a: RepTensor, b: RepTensor, c: RepTensor, m: int) -> RepTensor:
    """TruncPr(a * b + c, m).  On a per-party session the product's reshare is folded into
    the truncation: a * b + c goes through the dot tail (zero share + reshare + TruncPr, 2
    rounds instead of reshare + TruncPr's 2 after it), and a reveal merges the tail's
    second round with the reveal (parallel/party.py MulAddTail) -- the receiver only sums
    shares of the truncated value."""
    f = getattr(sess, "p_mul_add_deferred", None)
    if f is not None and 0 < m <= 63:
        r = f(a.plc, a, b, c, post_shift=m)
        if r is not None:
            return r
    return trunc_pr(sess, add(sess, mul(sess, a, b), c), m)


def mux(sess, s: RepTensor, x: RepTensor, y: RepTensor) -> RepTensor:
    """s ? x : y ; s is an arithmetic 0/1 sharing or a boolean bit sharing."""
    if s.kind == "bool":
        s = b2a(sess, s, x.bits)
    f = getattr(sess, "p_mux", None)
    if f is not None and x.kind == "arith" and y.kind == "arith":
        r = f(x.plc, s, x, y)  # the three steps in one kernel (same nonce, same shares)
        if r is not None:
            return RepTensor(x.plc, x.bits, "arith", r[0], r[1])
    return mul_add(sess, s, sub(sess, x, y), y)


def negate_where(sess, s: RepTensor, x: RepTensor) -> RepTensor:
    """x - 2 s x for an arithmetic 0/1 sharing s (|x| when s = [x < 0]): the product and the
    lincomb in one kernel on a stacked device session (same nonce, same shares)."""
    f = getattr(sess, "p_mux", None)
    if f is not None and s.kind == "arith" and x.kind == "arith":
        r = f(x.plc, s, x, x, absv=True)
        if r is not None:
            return RepTensor(x.plc, x.bits, "arith", r[0], r[1])
    return lincomb(sess, [(1, x), (-2, mul(sess, s, x))])


def abs_(sess, x: RepTensor) -> RepTensor:
    s = less_than_zero_arith(sess, x)
    return negate_where(sess, s, x)  # |x| = x - 2 s x


def relu(sess, x: RepTensor) -> RepTensor:
    s = less_than_zero_arith(sess, x)  # 1 if negative
    return sub(sess, x, mul(sess, s, x))


def ring_cast(sess, x: RepTensor, bits: int) -> RepTensor:
    """Z_2^128 -> Z_2^64 (share-wise truncation; valid for values that fit)."""
    return RepTensor(x.plc, bits, x.kind, sess.p("RingCast", x.plc, x.s0, bits=bits),
                     sess.p("RingCast", x.plc, x.s1, bits=bits))
