"""Per-party protocol steps shared by the layouts whose parties sit on different GPUs.

:class:`~moose_amd.parallel.cyclic.CyclicSession` (every GPU stacks one party of each of
three sessions) and :class:`~moose_amd.parallel.spmd.SPMDSession` (one party per process)
run the same per-party kernels (``csrc/rss_party.hip``); they differ only in which parties a
process hosts and how a message from party a to party b is routed.  A session provides

    party_exchange(plc, specs) -> {name: received tensor}

where ``specs`` is an ordered list of ``(name, a, b, tensor, like)``: message ``name`` goes
from party a to party b (``tensor`` = the payload on a process hosting a; ``like`` = the
payload's (shape, dtype) for the receiver to allocate, or the receiver's destination
tensor itself).  Every process walks the same
list in the same order, so the n-th message between two processes in one direction always
pairs with the n-th receive -- the role of the reference's rendezvous keys
(``moose/src/compilation/networking.rs``); no shape header travels.

Fixed-point dot tail (``rep.dot_trunc``): reference ``replicated/arith.rs:436-492`` (dot:
cross terms, zero share, reshare) followed by ``replicated/fixedpoint.rs:80-103`` ->
``additive/trunc.rs:114-170`` (TruncPr with dealer P2).  Here the reshare is folded into
TruncPr's first round (``rss_party.hip``): 2 rounds and 8 messages instead of 3 rounds and
9, with bitwise the same output shares.  Two schedule refinements on top:

* the dealer's messages (rt1, rm1) depend on keys and nonces only and go out before the
  GEMM (:func:`dealer_early`);
* round B can be left pending (:class:`RoundB`): a product that is revealed to the dealer
  next merges it with the reveal -- w0 and w1 go straight to P2 -- and otherwise it runs
  when the shares are first read (``protocols/replicated.py`` DeferredRep).
"""
from __future__ import annotations

import math

import torch

from moose_amd.ops import ring as R


def alias_exchange(specs):
    """party_exchange of a process hosting every party (stacked sessions): every
    message is the sender's buffer itself."""
    return {name: t for name, _a, _b, t, _like in specs}

# round A: (name, from party, to party); round B likewise
TAIL_A = (("m0", 0, 1), ("m1", 1, 0), ("z2_0", 2, 0), ("z2_1", 2, 1), ("rt1", 2, 1),
          ("rm1", 2, 1))
TAIL_B = (("w0", 0, 1), ("w1", 1, 0))


class DealerEarly:
    """The dealer's half of round A, done before the product exists (:func:`dealer_early`):
    P2's new shares already written into ``out0`` / ``out1``, P1's received rt1 / rm1."""

    __slots__ = ("out0", "out1", "rrt", "rrm", "stack", "event")

    def __init__(self, out0, out1, rrt, rrm):
        self.out0, self.out1, self.rrt, self.rrm = out0, out1, rrt, rrm
        self.stack = None  # the session's (s0, s1) tensors that out0 / out1 are views of
        self.event = None  # set when the dealer part ran on a side stream (wait before use)


def dealer_early(sess, plc, roles, like, bits, m, nonces, out0, out1, slots):
    """P2's TruncPr dealer messages of the dot tail (rt1, rm1 -> P1) depend on PRF keys and
    nonces only: computed and sent BEFORE the GEMM, they travel while it runs, and round A
    after the product carries only m0, m1 and z2 -- on the 2 -> 1 link 1 share tensor
    instead of 2.5.  ``like`` = (shape, dtype) of one component's product."""
    comp = {r: c for c, r in enumerate(roles)}
    n_el = math.prod(like[0]) // (2 if bits == 128 else 1)
    rt, rm = R.dot_tail_dealer(bits, m, roles, slots, nonces, out0, out1, n_el,
                               alloc=getattr(sess, "outbox", None))
    c2 = comp.get(2)
    got = sess.party_exchange(plc, [
        ("rt1", 2, 1, None if c2 is None else rt[c2], like),
        ("rm1", 2, 1, None if c2 is None else rm[c2], ((n_el,), torch.int64))])
    return DealerEarly(out0, out1, [got.get("rt1") if r == 1 else None for r in roles],
                       [got.get("rm1") if r == 1 else None for r in roles])


class RoundB:
    """Round B of the dot tail, not yet run (``dot_trunc_tail(..., defer=True)``): P0 and
    P1 hold w0 / w1, every other share is in place.  :meth:`finish` runs it (w0 <-> w1, then
    s1 of P0 and s0 of P1 = w0 + w1).  A reveal to the dealer P2 instead sends w0 and w1 to
    P2 (:meth:`reveal_to_dealer`): P2 holds z2, z0 and gets the third slot as w0 + w1, so
    the reshare round and the reveal round become ONE round of the same two messages (a
    product that is only revealed -- the benchmark's dot -- saves a round and a share
    tensor on the wire)."""

    def __init__(self, sess, plc, roles, w, out0, out1, bits, n_el, like):
        self.sess, self.plc, self.roles, self.w = sess, plc, roles, w
        self.out0, self.out1, self.bits, self.n_el, self.like = out0, out1, bits, n_el, like
        self.done = False
        t = next(x for x in out0 if x is not None)
        self.stream = R._stream_of(t)  # round A was issued here

    def _mine(self, party):
        c = {r: c for c, r in enumerate(self.roles)}.get(party)
        return None if c is None else self.w[c]

    def finish(self):
        if self.done:
            return
        self.done = True
        R._join(self.stream)
        sess, roles, like = self.sess, self.roles, self.like
        got = sess.party_exchange(self.plc, [("w0", 0, 1, self._mine(0), like),
                                             ("w1", 1, 0, self._mine(1), like)])
        other = [got.get("w1") if r == 0 else got.get("w0") if r == 1 else None for r in roles]
        dst = [self.out1[c] if r == 0 else self.out0[c] if r == 1 else None
               for c, r in enumerate(roles)]
        R.dot_tail_r2(self.w, other, dst, self.bits, roles, self.n_el)
        nb = math.prod(like[0]) * 8
        for a, b in ((0, 1), (1, 0)):
            sess.stats.record_send(self.plc.owners[a], self.plc.owners[b], nb)
        sess.stats.record_round(2 * nb)

    def reveal_to_dealer(self):
        """Open the product to P2: returns, for each hosted component playing P2, the four
        addends (z2, z0, w0, w1) of the value; None for other components.  The shares of
        P0 and P1 stay incomplete until something reads them (:meth:`finish`)."""
        sess, roles, like = self.sess, self.roles, self.like
        R._join(self.stream)
        got = sess.party_exchange(self.plc, [("w0", 0, 2, self._mine(0), like),
                                             ("w1", 1, 2, self._mine(1), like)])
        nb = math.prod(like[0]) * 8
        for a in (0, 1):
            sess.stats.record_send(self.plc.owners[a], self.plc.owners[2], nb)
        sess.stats.record_round(2 * nb)
        return [(self.out0[c], self.out1[c], got["w0"], got["w1"]) if r == 2 else None
                for c, r in enumerate(roles)]

    def reveal_to_member(self, j):
        """Open the (truncated) product to member P_j in ONE round after round A -- the
        reveal's round and round B merged, and only the value's own shares on the wire:

        * P2 (the dealer): P0 sends w0, P1 sends w1; P2 sums x2 + x0 + w0 + w1;
        * P0: P1 sends w1 + x2 (its round-B message plus its reveal message, summed);
          P0 sums x0 + w0 + (w1 + x2);
        * P1: P0 sends w0 + x0; P1 sums x2 + w1 + (w0 + x0).

        w0 + w1 = x1, so every receiver learns x0 + x1 + x2 -- the TruncPr'd value -- and
        nothing it would not learn from round B followed by the reveal.  Returns, for each
        hosted component playing P_j, the addends of the value; None for the others.  The
        shares stay pending (:meth:`finish` runs the ordinary round B if something reads
        them; the receiver already knows the value)."""
        if j == 2:
            return self.reveal_to_dealer()
        sess, roles, like, bits = self.sess, self.roles, self.like, self.bits
        R._join(self.stream)
        src = 1 - j  # the other non-dealer party
        mine = None
        c_src = {r: c for c, r in enumerate(roles)}.get(src)
        if c_src is not None:
            # P1 adds its x2 (out1), P0 its x0 (out0)
            own = self.out1[c_src] if src == 1 else self.out0[c_src]
            mine = R.binary("add", R.RT(self.w[c_src], bits),
                            R.RT(own.reshape(self.w[c_src].shape), bits),
                            alloc=getattr(sess, "outbox", None)).data
        got = sess.party_exchange(self.plc, [("wx", src, j, mine, like)])
        nb = math.prod(like[0]) * 8
        sess.stats.record_send(self.plc.owners[src], self.plc.owners[j], nb)
        sess.stats.record_round(nb)
        out = []
        for c, r in enumerate(roles):
            if r != j:
                out.append(None)
                continue
            keep = self.out0[c] if j == 0 else self.out1[c]  # x0 at P0, x2 at P1
            out.append((keep, self.w[c].reshape(keep.shape), got["wx"].reshape(keep.shape)))
        return out


class NoRoundB:
    """The deferred round of a process that hosts no party of the placement (SPMD
    outsiders): nothing to send, nothing to complete (a deferred truncation's nonces are
    drawn in step with the members: ``nonce_draw``)."""

    done = True

    def __init__(self, nonce_draw=None):
        self.nonce_draw = nonce_draw

    def finish(self):
        if self.nonce_draw is not None:
            draw, self.nonce_draw = self.nonce_draw, None
            draw()


def dot_trunc_tail(sess, plc, roles, cross, bits, m, nonces, out0, out1, slots, pre=None,
                   defer=False):
    """Zero share + reshare + TruncPr of the local cross products ``cross`` (one dense
    ring-``bits`` tensor per hosted component; component c plays party ``roles[c]``).
    Writes the new shares into ``out0`` / ``out1`` (dense per-component tensors, e.g. rows
    of a stack).  ``nonces`` = (zero share, r0, r1, t, m, z0, z2); ``slots`` = the key-slot
    pointers (own k_p, next k_{p+1}) of every component.  ``pre``: the dealer's part, done
    by :func:`dealer_early` (same out0 / out1).  ``defer``: return round B as a
    :class:`RoundB` instead of running it."""
    comp = {r: c for c, r in enumerate(roles)}
    n_el = math.prod(cross[0].shape) // (2 if bits == 128 else 1)
    box = getattr(sess, "outbox", None)  # where a thread receiver reads the messages
    msg, rt, rm = R.dot_tail_r0(cross, bits, m, roles, slots, nonces, out0, out1, n_el,
                                dealer=pre is None, alloc=box)

    def mine(party, arrs):
        c = comp.get(party)
        return None if c is None else arrs[c]

    like_rm = ((n_el,), torch.int64)
    like = (tuple(cross[0].shape), cross[0].dtype)
    payload = {"m0": mine(0, msg), "m1": mine(1, msg), "z2_0": mine(2, msg),
               "z2_1": mine(2, msg), "rt1": mine(2, rt), "rm1": mine(2, rm)}
    names = TAIL_A if pre is None else TAIL_A[:4]
    got = sess.party_exchange(plc, [(nm, a, b, payload[nm], like_rm if nm == "rm1" else like)
                                    for nm, a, b in names])
    rmk = [got.get("m1") if r == 0 else got.get("m0") if r == 1 else None for r in roles]
    rz = [got.get("z2_0") if r == 0 else got.get("z2_1") if r == 1 else None for r in roles]
    if pre is None:
        rrt = [got.get("rt1") if r == 1 else None for r in roles]
        rrm = [got.get("rm1") if r == 1 else None for r in roles]
    else:
        rrt, rrm = pre.rrt, pre.rrm
    w = R.dot_tail_r1(msg, rmk, rz, rrt, rrm, bits, m, roles, slots, nonces, out0, out1, n_el,
                      alloc=box)
    nb = cross[0].numel() * cross[0].element_size()
    record_tail_traffic(sess.stats, plc, nb, round_b=False)
    rb = RoundB(sess, plc, roles, w, out0, out1, bits, n_el, like)
    if defer:
        return rb
    rb.finish()
    return None


def record_tail_traffic(stats, plc, nb, round_b=True):
    """Messages of the folded dot tail (``nb`` bytes per share tensor): round A carries
    m0, m1, z2 (twice), rt1 and rm1 (a u64, half of a Z_2^128 element); round B w0, w1."""
    o = plc.owners
    for a, b, k in ((0, 1, 1), (1, 0, 1), (2, 0, 1), (2, 1, 2)):
        stats.record_send(o[a], o[b], nb, count=k)
    stats.record_send(o[2], o[1], nb // 2)
    stats.record_round(5 * nb + nb // 2)
    if not round_b:
        return
    for a, b in ((0, 1), (1, 0)):
        stats.record_send(o[a], o[b], nb)
    stats.record_round(2 * nb)


class PendingSums:
    """A level's round-2 sums not yet written (jobs_tail with ``defer``): this party's
    output rows o = w + received w, as regions the next level's round 0 reads through and
    writes (rss_jobs.hip Pend), or :meth:`flush` runs the round-2 kernel itself."""

    def __init__(self, jobs, L, bits, role, w, recv, regions):
        self.jobs, self.L, self.bits, self.role = jobs, L, bits, role
        self.w, self.recv, self.regions = w, recv, regions

    def flush(self):
        R.jobs_r2(self.jobs, self.L, self.bits, self.role, self.w, self.recv)


def _pending_regions(jobs, L, role, w, recv):
    """(o, a, b) flat views per job (o = P0's o1 / P1's o0 rows), or None when an output is
    not a dense block (then round 2 runs as its own kernel)."""
    regions, at = [], 0
    for j in jobs:
        o = j.o1 if role == 0 else j.o0
        n = j.rows * L
        per = w[0].numel()  # int64 words per element
        if o is None or not o.is_contiguous() or o.numel() != n * per or o.dtype != w.dtype:
            return None
        regions.append((o.reshape((n,) + tuple(w.shape[1:])), w[at:at + n], recv[at:at + n]))
        at += n
    return regions


def jobs_tail(sess, plc, role, jobs, L, bits, m, nonces, slots, pend=None, defer=False):
    """Zero share + reshare + TruncPr of the products ``jobs`` (ring.MulJob list) for ONE
    party of role ``role``: the dot tail's two rounds and three kernels (csrc/rss_jobs.hip)
    for all of them at once -- every job's cross terms computed inside round 0, the new
    shares written straight to the jobs' output rows.  ``nonces`` = the dot tail's seven.
    ``pend``: the previous level's :class:`PendingSums` (this round 0 completes them);
    ``defer``: return this level's round-2 sums as a PendingSums instead of running round 2
    (the caller hands them to the next level or flushes them before anything else reads)."""
    like = next(t for j in jobs for t in (j.o0, j.x0, j.a) if t is not None)
    box = getattr(sess, "outbox", None)
    alloc = (lambda shp: box(shp)) if box is not None else None
    msg, rt, rm = R.jobs_r0(jobs, L, bits, m, role, slots, nonces, like,
                            pend=pend.regions if pend is not None else None, alloc=alloc)
    n_el = sum(j.rows for j in jobs) * L
    like_t = ((n_el,) + ((2,) if bits == 128 else ()), torch.int64)
    like_rm = ((n_el,), torch.int64)
    payload = {"m0": msg if role == 0 else None, "m1": msg if role == 1 else None,
               "z2_0": msg if role == 2 else None, "z2_1": msg if role == 2 else None,
               "rt1": rt, "rm1": rm}
    got = sess.party_exchange(plc, [(nm, a, b, payload[nm], like_rm if nm == "rm1" else like_t)
                                    for nm, a, b in TAIL_A])
    rmk = got.get("m1") if role == 0 else got.get("m0") if role == 1 else None
    rz = got.get("z2_0") if role == 0 else got.get("z2_1") if role == 1 else None
    w = R.jobs_r1(jobs, L, bits, m, role, slots, nonces, msg, rmk, rz, got.get("rt1"),
                  got.get("rm1"), alloc=alloc)
    nb = n_el * (16 if bits == 128 else 8)
    record_tail_traffic(sess.stats, plc, nb, round_b=False)
    got = sess.party_exchange(plc, [("w0", 0, 1, w if role == 0 else None, like_t),
                                    ("w1", 1, 0, w if role == 1 else None, like_t)])
    out = None
    if role in (0, 1):
        recv = got["w1"] if role == 0 else got["w0"]
        regions = _pending_regions(jobs, L, role, w, recv) if defer else None
        if regions is not None:
            out = PendingSums(jobs, L, bits, role, w, recv, regions)
        else:
            R.jobs_r2(jobs, L, bits, role, w, recv)
    for a, b in ((0, 1), (1, 0)):
        sess.stats.record_send(plc.owners[a], plc.owners[b], nb)
    sess.stats.record_round(2 * nb)
    return out



class MulAddTail:
    """a * b + c for replicated a, b, c on a per-party session with the product's reshare
    pending (protocols/replicated.py mul_add_deferred): this party holds z, its zero-shared
    3-out-of-3 share of a * b.  :meth:`finish` is the reshare (z -> P_{p-1}) and the add;
    :meth:`reveal_to` opens a * b + c to a member P_j in ONE round instead of the reshare
    round plus the reveal: P_{j+1} sends z_{j+1} + c_{j+2}, P_{j+2} sends z_{j+2} + c_j
    (each its own z plus its second component), P_j sums z_j + c_{j+1} + both.

    ``post_shift`` = m > 0 (rep.mul_add_trunc): the value is TruncPr(a * b + c, m).  Then
    z + c0 (an additive share of the untruncated value) goes through the dot tail -- zero
    share + reshare + TruncPr, 2 rounds -- and a reveal merges the tail's round B with the
    reveal (:meth:`RoundB.reveal_to_member`): 2 rounds, and the receiver only ever holds
    shares of the TRUNCATED value (the reference reveals TruncPr'd shares too:
    replicated/convert.rs:280-313 after replicated/fixedpoint.rs:80-103)."""

    def __init__(self, sess, plc, z, c0, c1, bits, post_shift=0):
        self.sess, self.plc, self.z, self.c0, self.c1, self.bits = sess, plc, z, c0, c1, bits
        self.done = False
        self.rep = None  # the DeferredRep whose shares finish() completes
        self.post_shift = post_shift
        self._rb = None  # the truncating tail's round B (post_shift), once round A ran

    def _tail_round_a(self):
        """post_shift: the dot tail's round A on z + c0; the new shares land in the
        DeferredRep, round B stays pending (self._rb)."""
        from moose_amd.runtime.session import PV

        sess, bits = self.sess, self.bits
        v = R.binary("add", self.z, self.c0)
        nonces = tuple(sess.nonce(self.plc) for _ in range(7))
        s0, s1, self._rb = sess.party_dot_trunc(
            self.plc, PV(self.plc, R.RT(v.data.unsqueeze(0), bits)), self.post_shift, nonces,
            defer=True)
        self.rep._s0 = PV(self.plc, R.RT(s0.v.data[0], bits))
        self.rep._s1 = PV(self.plc, R.RT(s1.v.data[0], bits))

    def finish(self):
        if self.done:
            return
        self.done = True
        from moose_amd.runtime.session import PV

        if self.post_shift:
            if self._rb is None:
                self._tail_round_a()
            self._rb.finish()
            return
        zn = self.sess.shift(PV(self.plc, self.z), 1).v
        o0, o1 = R.binary2("add", self.z, self.c0, zn, self.c1)
        self.rep._s0, self.rep._s1 = PV(self.plc, o0), PV(self.plc, o1)

    def reveal_to(self, host):
        """The opened value at ``host`` (an Opened of its addends), None elsewhere; False
        when ``host`` is not a member (the caller finishes and reveals generically)."""
        plc = self.plc
        if host not in plc.owners:
            return False
        sess = self.sess
        j = plc.owners.index(host)
        idx = sess.party_index(plc)
        if self.post_shift:
            if self.done or self._rb is not None:
                return False  # shares already formed (or round A ran): the generic reveal
            self._tail_round_a()
            parts = self._rb.reveal_to_member(j)[0]
            # round B stays pending: a later reader runs it (finish)
            if idx != j:
                return None
            shape = self.z.data.shape
            return R.opened(*[R.RT(t.reshape(shape), self.bits) for t in parts])
        self.done = True
        like = (tuple(self.z.data.shape), self.z.data.dtype) if idx is not None else None
        mine = None
        if idx is not None and idx != j:
            # z + this party's second component (a message: into the session's outbox)
            mine = R.binary("add", self.z, self.c1, alloc=getattr(sess, "outbox", None)).data
        got = sess.party_exchange(plc, [("m1", (j + 1) % 3, j, mine if idx == (j + 1) % 3 else None,
                                         like),
                                        ("m2", (j + 2) % 3, j, mine if idx == (j + 2) % 3 else None,
                                         like)])
        nb = self.z.data.numel() * self.z.data.element_size() if idx is not None else 0
        for a in ((j + 1) % 3, (j + 2) % 3):
            sess.stats.record_send(plc.owners[a], host, nb)
        if idx != j:
            return None
        return R.opened(self.z, self.c1, R.RT(got["m1"], self.bits), R.RT(got["m2"], self.bits))
