"""Execution sessions: where party-local work runs and how shares move.

All MPC protocols (``moose_amd.protocols``) are written once against this API and run
under three sessions:

* :class:`StackedSession` -- all parties in one process on one device.  A party vector
  (``PV``) is a single tensor with a leading party axis of size 3, so one kernel launch
  does the local work of all three parties and a reshare is a roll of that axis.  This
  is the single-MI355X mode (and the CPU mode for tests); it plays the role of the
  reference's ``SyncSession``/``AsyncTestRuntime`` (``execution/synchronous.rs``,
  ``execution/asynchronous.rs:634-773``).
* :class:`moose_amd.parallel.spmd.SPMDSession` -- one process per party (one MI355X per
  party); every reshare is an RCCL send/recv over xGMI.
* :class:`moose_amd.compiler.symbolic.SymbolicSession` -- records host-level operations
  instead of executing them (compile-time lowering, reference ``execution/symbolic.rs``).

Vocabulary:

* ``HV`` -- a value living on one host (``host`` = role name).
* ``PV`` -- one component per party of a replicated placement ``plc``; component ``p``
  lives on ``plc.owners[p]``.

Keys: for every replicated placement the session holds k_0, k_1, k_2 (party p holds k_p
and k_{p+1}, so PRF(k_s) is computable by exactly the two holders of slot s) and k_all.
"""
from __future__ import annotations

import math
import os
import threading
from contextlib import contextmanager
from dataclasses import dataclass
from typing import Any
from typing import List
from typing import Optional

import numpy as np
import torch

from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ops import ring as R
from moose_amd.runtime import lanes as _lanes
from moose_amd.runtime.prims import PRIMS
from moose_amd.utils import telemetry


@dataclass
class HV:
    host: str
    v: Any


@dataclass
class PV:
    plc: ReplicatedPlacement
    v: Any


class Public:
    """Marks a value every party of a placement knows (no party axis)."""

    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v


# primitives whose eager implementation needs the session's device
_DEVICE_PRIMS = {"Fill", "Zeros", "Ones", "SampleSeeded", "Sample"}


def _nbytes(v):
    if isinstance(v, R.RT):
        if v.bits in (64, 128):  # without touching data (a lazy Encoded / Opened stays so)
            return v.numel() * (v.bits // 8)
        return v.data.numel() * v.data.element_size()
    if isinstance(v, torch.Tensor):
        return v.numel() * v.element_size()
    if isinstance(v, (bytes, bytearray)):
        return len(v)
    if type(v).__name__ == "KeyRef":
        return 16
    return 8


_SCOPE = threading.local()


@contextmanager
def nonce_scope(key: Optional[int]):
    """PRF nonces drawn in this thread come from scope ``key``'s own counter (Session.nonce);
    ``key`` >= 1 (None: the session-wide counter)."""
    prev = getattr(_SCOPE, "key", None)
    _SCOPE.key = key
    try:
        yield
    finally:
        _SCOPE.key = prev


class Session:
    """Common bookkeeping; see subclasses."""

    # input sharing: the owner's masked slot goes to P_{j+1} (1, the reference's direction,
    # replicated/convert.rs:74-90) or to P_{j+2} (2, mirrored); per owner role, set by a
    # layout that balances its links (parallel/cyclic.py default_layout)
    share_dirs: dict = {}

    def share_dir(self, plc, j) -> int:
        return self.share_dirs.get(plc.owners[j], 1)

    nb_party = 0

    def __init__(self, device="cpu", seed: Optional[int] = None):
        self.device = torch.device(device)
        self._nonces = {}
        self.seed = seed
        self.stats = telemetry.SessionStats()
        self._keys = {}
        self._rng = torch.Generator().manual_seed(seed) if seed is not None else None

    def nonce(self, plc=None) -> int:
        """Fresh PRF nonce of replicated placement ``plc``.  Every member of ``plc``
        executes every protocol step on ``plc`` in program order, so all members draw the
        same sequence; keeping one counter per placement keeps it aligned even when a
        party also works on other placements (SPMD execution).  Inside a
        :func:`nonce_scope` (the interpreter opens one per operation) the counter is the
        scope's own and the nonce is ``scope << 32 | n``: an operation's nonces do not
        depend on what ran before it or beside it, so independent operations can run
        interleaved (parallel/lockstep.py) with bitwise the shares of running them one by
        one."""
        sc = getattr(_SCOPE, "key", None)
        k = plc if sc is None else (sc, plc)
        n = self._nonces.get(k, 0) + 1
        self._nonces[k] = n
        return n if sc is None else (sc << 32) | n

    def _random_bytes(self, n=16) -> bytes:
        if self._rng is not None:
            return bytes(torch.randint(0, 256, (n,), generator=self._rng,
                                       dtype=torch.uint8).tolist())
        return os.urandom(n)

    def _attrs(self, prim, attrs):
        if prim in _DEVICE_PRIMS and "device" not in attrs:
            attrs = dict(attrs, device=self.device)
        return attrs


def _asym_applies(x, y) -> bool:
    """Whether a stacked product [3, M, K] . [3, K, N] takes the asymmetric local products:
    large products only (every dimension >= 256), a rule on the shape alone."""
    xs, ys = x.shape, y.shape
    return (len(xs) == 3 and len(ys) == 3 and xs[0] == 3 and ys[0] == 3 and x.bits in (64, 128)
            and min(xs[1], xs[2], ys[2]) >= 256)


class StackedSession(Session):
    """All three parties of every replicated placement on one device (module doc)."""

    nb_party = 1
    is_simulated = True

    # -- keys ------------------------------------------------------------------
    # Keys live in a device key table (runtime/keys.py): placement plc owns four slots
    # k0, k1, k2, k_all at self._keys[plc]; party p holds k_p and k_{p+1}.
    @property
    def keytable(self):
        kt = getattr(self, "_keytable", None)
        if kt is None:
            from moose_amd.runtime.keys import KeyTable

            kt = self._keytable = KeyTable(self.device, random_bytes=self._random_bytes)
        return kt

    def use_keytable(self, kt):
        """Run on a caller-provided key table (graph capture: a frozen, refreshed one)."""
        self._keytable = kt

    # rows per pipelined dot+TruncPr (protocols/replicated.dot_trunc); 1 = no pipelining
    pipeline_chunks = int(os.environ.get("MOOSEX_STACKED_CHUNKS", "1"))
    # the interpreter batches independent same-shape Dots into one launch sequence
    batch_dots = True

    def side_stream(self):
        """The HIP stream that pipelined protocol tails run on (created on first use)."""
        st = getattr(self, "_side", None)
        if st is None:
            st = self._side = torch.cuda.Stream(self.device)
        return st

    def setup(self, plc) -> int:
        base = self._keys.get(plc)
        if base is None:
            base = self.keytable.alloc(4)  # k0, k1, k2, k_all
            self._keys[plc] = base
        return base

    def key_ptr(self, plc, i) -> int:
        return self.keytable.ptr(self.setup(plc) + i)

    # -- host ops ----------------------------------------------------------------
    def h(self, prim, host, *args, **attrs):
        vals = []
        for a in args:
            if isinstance(a, HV):
                if a.host != host:
                    a = self.move(a, host)
                vals.append(a.v)
            elif isinstance(a, PV):
                raise TypeError("party vector passed to a host op")
            else:
                vals.append(a)
        return HV(host, PRIMS[prim].impl(0, *vals, **self._attrs(prim, attrs)))

    def move(self, x, host):
        if x.host != host:
            self.stats.record_send(x.host, host, _nbytes(x.v))
        return HV(host, x.v)

    def h_prf(self, plc, host, key_id, shape: HV, bits, nonce):
        """PRF(k_key_id, nonce) sampled on ``host`` (which must hold that key)."""
        ptr = self.key_ptr(plc, 3 if key_id == "all" else key_id)
        out = R.prf_expand_k(ptr, 1, nonce, tuple(shape.v), bits, self.device)
        return HV(host, R.RT(out.data[0], bits))

    def h_fresh_seed(self, host):
        from moose_amd.runtime.keys import KeyRef

        kt = self.keytable
        return HV(host, KeyRef(kt, kt.alloc(1)))

    # -- party vectors -------------------------------------------------------------
    def p(self, prim, plc, *args, **attrs):
        vals = []
        for a in args:
            if isinstance(a, PV):
                vals.append(a.v)
            elif isinstance(a, Public):
                v = a.v
                if prim in ("Dot", "Concat"):
                    v = _stack3(v)
                vals.append(v)
            elif isinstance(a, HV):
                raise TypeError("host value passed to a party-vector op; use public()")
            else:
                vals.append(a)
        return PV(plc, PRIMS[prim].impl(1, *vals, **self._attrs(prim, attrs)))

    def public(self, plc, value):
        return Public(value)

    def shift(self, x, k=1):
        """Component p <- component p+k (one communication round)."""
        self.stats.record_round(_nbytes(x.v))
        v = x.v
        if isinstance(v, R.RT):
            return PV(x.plc, R.RT(torch.roll(v.data, -k, dims=0), v.bits))
        return PV(x.plc, torch.roll(v, -k, dims=0))

    def take(self, x, i):
        v = x.v
        if isinstance(v, R.RT):
            return HV(x.plc.owners[i], R.RT(v.data[i], v.bits))
        return HV(x.plc.owners[i], v[i])

    def gather(self, plc, xs):
        for i, x in enumerate(xs):
            if x.host != plc.owners[i]:
                self.stats.record_send(x.host, plc.owners[i], _nbytes(x.v))
        vs = [x.v for x in xs]
        if isinstance(vs[0], R.RT):
            return PV(plc, R.RT(torch.stack([v.data for v in vs]), vs[0].bits))
        return PV(plc, torch.stack(vs))

    def p_public_slot(self, plc, value, slot, bits):
        v = value if isinstance(value, R.RT) else R.fill((), int(value), bits, self.device)
        d = torch.zeros((3,) + tuple(v.data.shape), dtype=v.data.dtype, device=self.device)
        d[slot] = v.data
        return PV(plc, R.RT(d, bits))

    def p_apply_at(self, prim, plc, x, which, c):
        """Apply ``prim(component, c)`` on party ``which`` only."""
        v = x.v
        op = {"Add": "add", "Sub": "sub", "Xor": "xor", "And": "and", "Mul": "mul"}.get(prim)
        if op is not None and isinstance(c, R.RT) and c.bits == v.bits and v.bits in (1, 64, 128):
            if R._slot_operand_ok(v, c):  # scalar, slot-shaped or trailing-axes vector
                return PV(plc, R.binary_slot(op, v, c, which))  # one kernel
        part = PRIMS[prim].impl(0, R.RT(v.data[which], v.bits), c)
        d = v.data.clone() if part.data.shape == v.data.shape[1:] else None
        if d is None:  # broadcasting changed the shape
            shp = (3,) + tuple(part.data.shape)
            d = v.data.expand(shp).clone()
        d[which] = part.data
        return PV(plc, R.RT(d, v.bits))

    # -- share pairs: both share vectors of a share-wise op in one launch ----------------
    _PAIR_BIN = {"Add": "add", "Sub": "sub", "Xor": "xor", "And": "and", "Mul": "mul"}

    # per-party primitives that run over a pair-stacked base (every slot independent)
    _PAIR_SLOTWISE = ("WeightedSum", "BitExtract", "BitSplit", "Slice")
    # slot-wise with one public operand, the same for both share vectors
    _PAIR_SLOTWISE_PUB = ("MulLeading",)

    @staticmethod
    def _pair_base(v0, v1):
        """(base, n, off): when the two share vectors are views of ONE buffer -- a share-pair
        ring (s1 = s0 + 1 slot: 4 slots) or adjacent halves of a pair allocation (s1 = s0 +
        3 slots: 6 slots) -- the buffer's slots as one [n, ...] tensor and s1's offset in
        slots; None otherwise."""
        if not (isinstance(v0, R.RT) and isinstance(v1, R.RT)):
            return None
        d0, d1 = v0.data, v1.data
        if (d0.dim() < 1 or d0.shape != d1.shape or d0.stride() != d1.stride()
                or d0.shape[0] != 3 or d0.dtype != d1.dtype or d0.stride(0) <= 0
                or d0.untyped_storage().data_ptr() != d1.untyped_storage().data_ptr()):
            return None
        step = d0.stride(0) * d0.element_size()
        off = d1.data_ptr() - d0.data_ptr()
        if off == step:
            n, o = 4, 1
        elif off == 3 * step:
            n, o = 6, 3
        else:
            return None
        try:
            base = d0.as_strided((n,) + tuple(d0.shape[1:]), d0.stride())
        except RuntimeError:  # not inside one storage
            return None
        return R.RT(base, v0.bits), n, o

    def p_pair(self, prim, plc, a, b=None, **attrs):
        """(prim(a[0], b[0]), prim(a[1], b[1])) as one kernel when both are ring tensors of
        64/128 bits (Neg / Shl / the binary ring ops), or for a slot-wise primitive when the
        pair is one buffer (``_pair_base``); None -> caller issues two ops."""
        pub = (b is not None and prim in self._PAIR_SLOTWISE_PUB and b[0] is b[1]
               and isinstance(b[0], Public))
        if (b is None and prim in self._PAIR_SLOTWISE) or pub:
            pb = self._pair_base(a[0].v, a[1].v)
            if pb is None:
                return None
            base, n, o = pb
            extra = (b[0].v,) if pub else ()
            out = PRIMS[prim].impl(1, base, *extra, **self._attrs(prim, attrs))
            return (PV(plc, R.RT(out.data[0:3], out.bits)),
                    PV(plc, R.RT(out.data[o:o + 3], out.bits)))
        v0, v1 = a[0].v, a[1].v
        if not (isinstance(v0, R.RT) and isinstance(v1, R.RT)) or v0.bits not in (64, 128):
            return None
        if b is None:
            if prim == "Neg":
                o0, o1 = R.unary2("neg", v0, v1)
            elif prim == "Shl":
                o0, o1 = R.unary2("shl", v0, v1, attrs["amount"])
            else:
                return None
            return PV(plc, o0), PV(plc, o1)
        op = self._PAIR_BIN.get(prim)
        if op is None:
            return None
        w = [x.v for x in b]
        if not all(isinstance(t, R.RT) and t.bits == v0.bits for t in w):
            return None
        o0, o1 = R.binary2(op, v0, w[0], v1, w[1])
        return PV(plc, o0), PV(plc, o1)

    def p_dot_public_pair(self, plc, x0, x1, c):
        """rep.dot_public (x . c, c public) for both share vectors: when they are the two
        views of one share-pair ring buffer (s0 = buf[0:3], s1 = buf[1:4]), ONE product of
        the buffer's four slots with c, read in place by every slot, whose result is again
        a ring buffer; otherwise one launch per share vector, still without copying c per
        party.  None -> the generic path."""
        v0, v1, cv = x0.v, x1.v, c.v
        if not (isinstance(v0, R.RT) and isinstance(v1, R.RT) and isinstance(cv, R.RT)):
            return None
        if self.device.type != "cuda" or v0.bits not in (64, 128) or cv.bits != v0.bits:
            return None
        d0, d1 = v0.data, v1.data
        el = 2 if v0.bits == 128 else 1
        if (d0.dim() >= 2 and d0.shape == d1.shape and d0.stride() == d1.stride()
                and d0.shape[0] == 3
                and d1.data_ptr() - d0.data_ptr() == d0.stride(0) * d0.element_size()
                and d0.stride(0) % el == 0):
            buf = R.RT(d0.as_strided((4,) + tuple(d0.shape[1:]), d0.stride()), v0.bits)
            o = R.dot_slots(buf, cv)
            if o is not None:
                return PV(plc, R.RT(o.data[0:3], o.bits)), PV(plc, R.RT(o.data[1:4], o.bits))
        o0, o1 = R.dot_slots(v0, cv), R.dot_slots(v1, cv)
        if o0 is None or o1 is None:
            return None
        return PV(plc, o0), PV(plc, o1)

    def p_b2a_prep(self, plc, b, ring_bits):
        """rep.b2a's local steps in one kernel (device): (P0's a = b_0 ^ b_1 as a ring
        value, the trivial sharing of b_2 as a (s0, s1) pair); None -> the generic steps."""
        if self.device.type != "cuda":
            return None
        v0, v1 = b.s0.v, b.s1.v
        if not (isinstance(v0, R.RT) and isinstance(v1, R.RT)) or v0.bits != 1:
            return None
        r = R.b2a_prep3(v0, v1, ring_bits)
        if r is None:
            return None
        a, o0, o1 = r
        return HV(plc.owners[0], a), PV(plc, o0), PV(plc, o1)

    def p_b2a(self, plc, b, ring_bits):
        """The whole of rep.b2a in one kernel (device, fused session): the same nonces in
        the same order (share: n1, na; mul: nmul) and the same traffic records as the
        share + mul + lincomb steps, so the same shares.  None -> those steps."""
        if self.device.type != "cuda" or not getattr(self, "fused", False) \
                or os.environ.get("MOOSEX_B2A_FUSED", "1") == "0":
            return None
        v0, v1 = b.s0.v, b.s1.v
        if not (isinstance(v0, R.RT) and isinstance(v1, R.RT)) or v0.bits != 1 \
                or ring_bits not in (64, 128) or not v0.data.is_cuda \
                or v0.data.dtype != torch.uint8 or v1.data.dtype != torch.uint8 \
                or v0.data.shape != v1.data.shape or v0.data.shape[0] != 3:
            return None  # (R.b2a3's own conditions, checked before any nonce is drawn)
        d = self.share_dir(plc, 0)
        n1, _na, nmul = self.nonce(plc), self.nonce(plc), self.nonce(plc)
        o0, o1 = R.b2a3(v0, v1, ring_bits, self.key_ptr(plc, 0), d == 2, n1, nmul)
        nb = math.prod(v0.shape[1:]) * (ring_bits // 8)
        self.stats.record_send(plc.owners[0], plc.owners[d % 3], nb)
        self.stats.record_round(3 * nb)
        return PV(plc, o0), PV(plc, o1)

    def p_b2a_planes(self, plc, b, start, count, ring_bits):
        """rep.b2a of the bit planes start..start+count-1 of the packed boolean sharing
        ``b`` (BitSplit + b2a) in one kernel: the b2a's nonces and traffic records as
        p_b2a draws and records them.  None -> the two steps."""
        if self.device.type != "cuda" or not getattr(self, "fused", False) \
                or os.environ.get("MOOSEX_B2A_FUSED", "1") == "0":
            return None
        v0, v1 = b.s0.v, b.s1.v
        if not (isinstance(v0, R.RT) and isinstance(v1, R.RT)) or v0.bits != ring_bits \
                or v0.bits not in (64, 128) or v1.shape != v0.shape or v0.shape[0] != 3 \
                or start < 0 or count < 1 or start + count > v0.bits:
            return None
        d = self.share_dir(plc, 0)
        n1, _na, nmul = self.nonce(plc), self.nonce(plc), self.nonce(plc)
        o0, o1 = R.b2a3_planes(v0, v1, start, count, self.key_ptr(plc, 0), d == 2, n1, nmul)
        nb = count * math.prod(v0.shape[1:]) * (ring_bits // 8)
        self.stats.record_send(plc.owners[0], plc.owners[d % 3], nb)
        self.stats.record_round(3 * nb)
        return PV(plc, o0), PV(plc, o1)

    def p_mul_leading_add(self, plc, x0, x1, c, cadd):
        """MulLeading of a share pair by the public vector ``c`` then add_public of the scalar
        ``cadd`` (slot 0 of s0, slot 2 of s1), one launch over the pair buffer (no nonce, no
        traffic).  None -> the two steps."""
        if self.device.type != "cuda" or not getattr(self, "fused", False):
            return None
        pb = self._pair_base(x0.v, x1.v)
        if pb is None:
            return None
        base, k, o = pb
        r = R.mul_leading_add(base, c, 1, cadd, (0, o + 2))
        if r is None:
            return None
        return PV(plc, R.RT(r.data[0:3], r.bits)), PV(plc, R.RT(r.data[o:o + 3], r.bits))

    def p_mux(self, plc, s, x, y, absv=False):
        """rep.mux(s, x, y) = s * (x - y) + y (arithmetic) in one kernel: the product's one
        nonce and its round as rep.mul draws and records them.  ``absv``: x - 2 s x
        (rep.lincomb of x and mul(s, x); y is x).  None -> the three steps."""
        if self.device.type != "cuda" or not getattr(self, "fused", False):
            return None
        vs = [t.v for t in (s.s0, s.s1, x.s0, x.s1, y.s0, y.s1)]
        if not all(isinstance(v, R.RT) for v in vs) or vs[0].bits not in (64, 128) or any(
                v.bits != vs[0].bits or v.shape != vs[0].shape for v in vs) \
                or len(vs[0].shape) < 1 or vs[0].shape[0] != 3 or not vs[0].data.is_cuda:
            return None
        r = R.mux3(*vs, self.key_ptr(plc, 0), self.nonce(plc), absv=absv)
        if r is None:  # a nonce is drawn: never fall back silently
            raise RuntimeError("mux3 declined after its checks")
        self.stats.record_round(_nbytes(r[0]))
        return PV(plc, r[0]), PV(plc, r[1])

    def p_sign_arith(self, plc, x, width=None):
        """rep.b2a(rep.msb(x)) in one kernel: p_bit_decompose's work, then the top bit's
        b2a (its sharing nonces n1', na' and product nonce nmul' after the decomposition's,
        as the two protocol steps draw them).  ``width`` (a bound on the value's bits) is
        not needed here: the whole-word chain is one kernel.  None -> the steps."""
        return self.p_bit_decompose(plc, x, sign=True)

    def p_bit_decompose(self, plc, x, sign=False, width=None):
        """The whole of rep.bit_decompose in one kernel (device, fused session, latency
        sizes): the nonces in the generic order (share: n1, na; the adder's AND: nmul; one
        per level) and the same traffic records, so the same shares.  None -> the steps."""
        if self.device.type != "cuda" or not getattr(self, "fused", False) \
                or os.environ.get("MOOSEX_BITDEC_FUSED", "1") == "0":
            return None
        v0, v1 = x.s0.v, x.s1.v
        if not (isinstance(v0, R.RT) and isinstance(v1, R.RT)) or v0.bits not in (64, 128) \
                or v1.bits != v0.bits or v0.shape != v1.shape or not v0.data.is_cuda \
                or len(v0.shape) < 1 or v0.shape[0] != 3:
            return None
        bits = v0.bits
        n = math.prod(v0.shape[1:])
        if n > 65536:
            return None
        d = self.share_dir(plc, 0)
        n1, _na, nmul = self.nonce(plc), self.nonce(plc), self.nonce(plc)
        nonces = [self.nonce(plc) for _ in range(bits.bit_length() - 1)]
        sn = None
        if sign:
            n1b, _nab, nmulb = self.nonce(plc), self.nonce(plc), self.nonce(plc)
            sn = (n1b, nmulb)
        o0, o1 = R.bitdec3(v0, v1, self.key_ptr(plc, 0), d == 2, n1, nmul, nonces, sn)
        nb = n * (bits // 8)
        self.stats.record_send(plc.owners[0], plc.owners[d % 3], nb)  # the sharing of y
        self.stats.record_round(3 * nb)  # the adder's AND
        dd = 1
        for _ in nonces:  # the chain's rounds
            self.stats.record_round(3 * nb * (2 if 2 * dd < bits else 1))
            dd *= 2
        if sign:  # the b2a of the top bit: its sharing and its product round
            self.stats.record_send(plc.owners[0], plc.owners[d % 3], nb)
            self.stats.record_round(3 * nb)
        return PV(plc, o0), PV(plc, o1)

    def p_from_slot_holders(self, plc, slot, x_h0, x_h1, like):
        """rep.from_slot_holders in one kernel (None -> generic path)."""
        v0, v1 = x_h0.v, x_h1.v
        if not (isinstance(v0, R.RT) and isinstance(v1, R.RT)) or v0.bits not in (64, 128) \
                or v1.shape != v0.shape or tuple(v0.shape) != tuple(like.v.shape[1:]):
            return None
        o = plc.owners
        h0, h1 = slot, (slot - 1) % 3
        if x_h0.host != o[h0] or x_h1.host != o[h1]:
            return None
        a, b = R.slot_place2(v0, v1, h0, h1)
        return PV(plc, a), PV(plc, b)

    def p_reveal(self, x, host):
        """Reveal to a member P_j: its two shares plus the third (from P_{j+1}) summed in one
        kernel; None for outsiders (generic)."""
        if host not in x.plc.owners:
            return None
        v0, v1 = x.s0.v, x.s1.v
        if not (isinstance(v0, R.RT) and isinstance(v1, R.RT)):
            return None
        j = x.plc.owners.index(host)
        j1 = (j + 1) % 3
        self.stats.record_send(x.plc.owners[j1], host, _nbytes(v1) // 3)
        return HV(host, R.opened(R.RT(v0.data[j], v0.bits), R.RT(v1.data[j], v1.bits),
                                 R.RT(v1.data[j1], v1.bits)))

    def p_add_n(self, plc, xs):
        """Sum of replicated values ``xs`` [(PV s0, PV s1)] in one kernel when they are evenly
        spaced views of one stack (e.g. the products of a batched Dot); None otherwise."""
        v0, v1 = [a.v for a, _ in xs], [b.v for _, b in xs]
        if len(xs) < 2 or not all(isinstance(t, R.RT) for t in v0 + v1):
            return None
        if v0[0].bits not in (64, 128):
            return None
        r = R.sum_views2(v0, v1)
        if r is None:
            return None
        return PV(plc, r[0]), PV(plc, r[1])

    def p_lincomb(self, plc, terms, const=None):
        """sum_t k_t * x_t (+ public const on party 0's share) for 64/128-bit replicated
        values of one shape, one kernel; ``terms`` = [(k, PV s0, PV s1)].  None -> the
        caller composes the share-wise ops."""
        if not 1 <= len(terms) <= 3:
            return None
        vs = [(k, a.v, b.v) for k, a, b in terms]
        v0 = vs[0][1]
        if not all(isinstance(a, R.RT) and isinstance(b, R.RT) for _, a, b in vs):
            return None
        if v0.bits not in (64, 128) or any(
                a.bits != v0.bits or b.bits != v0.bits or a.shape != v0.shape or b.shape != v0.shape
                for _, a, b in vs):
            return None
        if const is not None and not (isinstance(const, R.RT) and const.bits == v0.bits
                                      and R._slot_operand_ok(v0, const)):
            return None
        o0, o1 = R.lincomb2(vs, const, 0, 2)
        return PV(plc, o0), PV(plc, o1)

    def p_apply_at2(self, prim, plc, x0, x1, which0, which1, c):
        """p_apply_at on both share vectors in one kernel (None if not applicable)."""
        op = self._PAIR_BIN.get(prim)
        v0, v1 = x0.v, x1.v
        if (op is None or not isinstance(c, R.RT) or c.bits != v0.bits
                or v0.bits not in (64, 128) or v1.shape != v0.shape
                or not R._slot_operand_ok(v0, c)):
            return None
        o0, o1 = R.binary_slot2(op, v0, v1, c, which0, which1)
        return PV(plc, o0), PV(plc, o1)

    # -- stacked rows (device): build [3, n, ...] stacks in place instead of concat/slice --
    def p_rows_alloc(self, x, n):
        """A [3, n, *shape] stack whose row 0 is x (rows 1.. written later)."""
        v = x.v
        d = torch.empty((v.data.shape[0], n) + tuple(v.data.shape[1:]), dtype=v.data.dtype,
                        device=v.data.device)
        d[:, 0].copy_(v.data)
        return PV(x.plc, R.RT(d, v.bits))

    def p_rows_alloc_pair(self, x0, x1, n):
        """p_rows_alloc for both share vectors of a replicated value: when they are the two
        views of one share-pair ring buffer, ONE [4, n, ...] ring stack whose row 0 is
        filled by one copy of the buffer's four slots (P0 = stack[0:3], P1 = stack[1:4];
        the kernels that write later rows see a ring pair and write four slots)."""
        v0, v1 = x0.v, x1.v
        pb = self._pair_base(v0, v1)
        if pb is not None and v0.data[0].is_contiguous():
            base, k, o = pb
            d0 = v0.data
            st = torch.empty((k, n) + tuple(d0.shape[1:]), dtype=d0.dtype, device=d0.device)
            st[:, 0].copy_(base.data)  # one copy for both share vectors
            return PV(x0.plc, R.RT(st[0:3], v0.bits)), PV(x1.plc, R.RT(st[o:o + 3], v1.bits))
        return self.p_rows_alloc(x0, n), self.p_rows_alloc(x1, n)

    def p_rows_view(self, x, r0, r1):
        return PV(x.plc, R.RT(x.v.data[:, r0:r1], x.v.bits))

    def p_rows_bcast(self, x, r, m):
        d = x.v.data[:, r:r + 1]
        return PV(x.plc, R.RT(d.expand((d.shape[0], m) + tuple(d.shape[2:])), x.v.bits))

    def p_rows_write(self, x, r0, src):
        s = src.v.data
        x.v.data[:, r0:r0 + s.shape[1]].copy_(s)

    def p_repeat0(self, x, k):
        """k copies of a party vector on a new axis after the party axis, as a stride-0
        view (consumers that need memory materialise it; the batched GEMM does not)."""
        v = x.v
        d = v.data.unsqueeze(1)
        return PV(x.plc, R.RT(d.expand((d.shape[0], k) + tuple(d.shape[2:])), v.bits))

    def p_stack2(self, a, b):
        return PV(a.plc, R.RT(torch.stack([a.v.data, b.v.data], dim=1), a.v.bits))

    def p_unstack2(self, x):
        return (PV(x.plc, R.RT(x.v.data[:, 0], x.v.bits)),
                PV(x.plc, R.RT(x.v.data[:, 1], x.v.bits)))

    # -- fused RSS kernels -----------------------------------------------------------
    def p_cross(self, kind, plc, x0, x1, y0, y1, zero_share=True):
        """Party p: x0*y0 + x0*y1 + x1*y0 (+ alpha_p with sum alpha = 0), one kernel."""
        x1v = x1.v if x1 is not None else None
        y1v = y1.v if y1 is not None else None
        if not zero_share:
            return PV(plc, R.rss_cross(kind, x0.v, x1v, y0.v, y1v, None, self.nonce(plc), 3))
        out = R.rss_cross_k(kind, x0.v, x1v, y0.v, y1v, self.key_ptr(plc, 0), 3,
                            self.nonce(plc), 3)
        return PV(plc, out)

    def p_mul_reshare(self, kind, plc, x0, x1, y0, y1):
        """Both shares of x*y after the reshare, in one kernel (protocol of rep.mul:
        cross terms + zero share, then z_p -> P_{p-1})."""
        s0, s1 = R.rss_mul3_k(kind, x0.v, x1.v, y0.v, y1.v, self.key_ptr(plc, 0),
                              self.nonce(plc))
        self.stats.record_round(_nbytes(s0))
        return PV(plc, s0), PV(plc, s1)

    def p_mul_trunc(self, plc, x0, x1, y0, y1, m, out=None):
        """rep.mul + rep.trunc_pr (arith) in one kernel (device: the latency form for small
        launches, the throughput form above); None -> the caller runs the two protocol
        steps.  Draws the same nonces in the same order as the two steps."""
        if self.device.type != "cuda":
            return None
        v = [t.v for t in (x0, x1, y0, y1)]
        if not all(isinstance(t, R.RT) for t in v) or v[0].bits not in (64, 128):
            return None
        if any(t.shape != v[0].shape for t in v):
            return None
        if any(not t.data.is_contiguous() and R._party_view(t) is None for t in v):
            return None
        if out is not None:
            o = [t.v.data for t in out]
            if not (tuple(out[0].v.shape) == tuple(v[0].shape) == tuple(out[1].v.shape)
                    and o[0].stride(0) == o[1].stride(0) and o[0][0].is_contiguous()
                    and o[1][0].is_contiguous()):
                return None
        nmul = self.nonce(plc)
        nonces = tuple(self.nonce(plc) for _ in range(6))
        outs = None if out is None else (out[0].v, out[1].v)
        r = R.mul_trunc3_k(*v, self.key_ptr(plc, 0), nmul, m, nonces, out=outs)
        if r is None:  # cannot happen after the checks above; keep the protocol honest
            raise RuntimeError("mul_trunc3 declined after its checks")
        from moose_amd.parallel.party import record_tail_traffic

        # the messages of the per-party protocol (reshare folded into TruncPr, 2 rounds)
        record_tail_traffic(self.stats, plc, _nbytes(r[0]) // 3)
        return PV(plc, r[0]), PV(plc, r[1])

    def p_mul_trunc2(self, plc, jobs):
        """Two independent p_mul_trunc products [(x0, x1, y0, y1, m, out)] in ONE launch
        (k_mul_trunc3_lat2), the nonces drawn in the order two p_mul_trunc calls draw them
        (so the shares are the same).  None -> the caller runs them one by one."""
        if self.device.type != "cuda" or len(jobs) != 2:
            return None
        args = []
        for x0, x1, y0, y1, m, out in jobs:
            v = [t.v for t in (x0, x1, y0, y1)]
            if not all(isinstance(t, R.RT) for t in v) or not m:
                return None
            o = None if out is None else (out[0].v, out[1].v)
            if R._mt3_args(*v, out=o) is None:
                return None
            args.append((v, m, o))
        bits = args[0][0][0].bits
        n_max = 8192 * (1 if bits == 128 else 2)
        if any(math.prod(a[0][0].shape) // 3 > n_max for a in args):
            return None
        batched = []
        for v, m, o in args:
            nmul = self.nonce(plc)
            nonces = tuple(self.nonce(plc) for _ in range(6))
            batched.append((*v, nmul, m, nonces, o))
        r = R.mul_trunc3_k2(batched, self.key_ptr(plc, 0))
        if r is None:  # nonces are drawn: never fall back silently
            raise RuntimeError("mul_trunc3 x2 declined after its checks")
        from moose_amd.parallel.party import record_tail_traffic

        out = []
        for o0, o1 in r:
            record_tail_traffic(self.stats, plc, _nbytes(o0) // 3)
            out.append((PV(plc, o0), PV(plc, o1)))
        return out

    def p_cross_plain(self, kind, plc, x0, x1, y0, y1):
        """The parties' cross terms with no zero share and no nonce drawn (the per-party
        tail, rep.mul_trunc on the host, adds the zero share)."""
        return PV(plc, R.rss_cross(kind, x0.v, x1.v, y0.v, y1.v, None, 0, 3))

    def p_zs_trunc(self, plc, z, m):
        """The tail of a fixed-point dot in one kernel (device): rep.dot's zero share and
        reshare of the local products ``z`` and rep.trunc_pr of the result -- the same
        nonces in the same order as the two steps, so the same shares.  None on the host."""
        if self.device.type != "cuda" or z.v.bits not in (64, 128) or not m:
            return None
        nmul = self.nonce(plc)
        nonces = tuple(self.nonce(plc) for _ in range(6))
        r = R.zs_trunc3_k(z.v, self.key_ptr(plc, 0), nmul, m, nonces)
        if r is None:  # nonces are drawn: never fall back silently
            raise RuntimeError("zs_trunc3 declined on a device session")
        from moose_amd.parallel.party import record_tail_traffic

        # the messages of the per-party protocol (reshare folded into TruncPr, 2 rounds)
        record_tail_traffic(self.stats, plc, _nbytes(r[0]) // 3)
        return PV(plc, r[0]), PV(plc, r[1])

    def p_zs_trunc_rows(self, plc, z, m, buf4, r0):
        """p_zs_trunc of a row block of a pipelined product (rep.dot_trunc with
        ``pipeline_chunks`` > 1): the new shares written into rows [r0, r0 + rows) of the
        result's [4, M, N] share-pair ring buffer ``buf4``.  The chunk is its own protocol
        instance (its own nonces)."""
        nmul = self.nonce(plc)
        nonces = tuple(self.nonce(plc) for _ in range(6))
        R.zs_trunc3_rows(z.v, self.key_ptr(plc, 0), nmul, m, nonces, buf4, r0)
        from moose_amd.parallel.party import record_tail_traffic

        record_tail_traffic(self.stats, plc, _nbytes(z.v) // 3)

    def party_exchange(self, plc, specs):
        """Every party is local: a per-party message is the sender's buffer."""
        return {name: t for name, _a, _b, t, _like in specs}

    def party_dot_trunc(self, plc, v, m, nonces, out=None):
        """rep.dot_trunc's tail with the per-party kernels (reshare folded into TruncPr's
        first round, parallel/party.py): the host path; a device session runs the whole tail
        as one kernel (p_zs_trunc), which gives the same shares."""
        from moose_amd.parallel import party

        bits = v.v.bits
        data = v.v.data.contiguous()
        if out is not None:  # party vectors (row views of a stack) or raw tensors
            s0, s1 = (o.v.data if isinstance(o, PV) else o for o in out)
        else:
            s0, s1 = torch.empty_like(data), torch.empty_like(data)
        slots = [self.key_ptr(plc, q) for p in range(3) for q in (p, (p + 1) % 3)]
        party.dot_trunc_tail(self, plc, [0, 1, 2], [data[c] for c in range(3)], bits, m,
                             nonces, [s0[c] for c in range(3)], [s1[c] for c in range(3)], slots)
        return PV(plc, R.RT(s0, bits)), PV(plc, R.RT(s1, bits))

    def p_ks_adder(self, plc, g0, g1, p0, p1, bits, sum_out=False):
        """rep.binary_adder's carry chain, all log2(bits) levels in one kernel (device
        sessions); the nonces of the per-level chain, in its order.  ``sum_out``: the
        adder's sum p ^ (g << 1) instead of the carries.  None on the host."""
        if self.device.type != "cuda":
            return None
        nlev = bits.bit_length() - 1
        nonces = [self.nonce(plc) for _ in range(nlev)]
        o0, o1 = R.ks_adder3_k(g0.v, g1.v, p0.v, p1.v, self.key_ptr(plc, 0), nonces,
                               sum_out=sum_out)
        d = 1
        for _ in range(nlev):  # the rounds of the chain it replaces
            self.stats.record_round(_nbytes(o0) * (2 if 2 * d < bits else 1))
            d *= 2
        return PV(plc, o0), PV(plc, o1)

    def p_ks_level(self, plc, g0, g1, p0, p1, d, both):
        """One Kogge-Stone level of rep.binary_adder (AND(s) + reshare + xor) in one
        kernel; consumes the one nonce of the generic level's AND round."""
        og0, og1, op0, op1 = R.ks_level3_k(g0.v, g1.v, p0.v, p1.v, d, both,
                                           self.key_ptr(plc, 0), self.nonce(plc))
        self.stats.record_round(_nbytes(og0) * (2 if both else 1))
        if not both:
            return PV(plc, og0), PV(plc, og1), None, None
        return PV(plc, og0), PV(plc, og1), PV(plc, op0), PV(plc, op1)

    def p_zero_share_reshare(self, plc, z, kind="arith"):
        """z_p + alpha_p, reshared (the tail of rep.dot), in one kernel."""
        s0, s1 = R.rss_mul3_k(kind, z.v, None, None, None, self.key_ptr(plc, 0),
                              self.nonce(plc))
        self.stats.record_round(_nbytes(s0))
        return PV(plc, s0), PV(plc, s1)

    def p_dot_zs_reshare(self, plc, x0, x1, y0, y1, kind):
        """rep.dot's local part + zero share + reshare with the zero-share keystreams
        generated on a side stream WHILE the MFMA GEMM runs (AES is VALU/LDS work, the
        GEMM is MFMA work; both fit on a CU).  Same nonce and values as
        p_dot_cross + p_zero_share_reshare.  Returns None when not applicable."""
        if (kind != "arith" or self.device.type != "cuda" or os.environ.get(
                "MOOSEX_OVERLAP_ZS", "0") == "0"):  # opt-in until measured
            return None
        shp, yshp = tuple(x0.v.shape), tuple(y0.v.shape)
        if len(shp) != 3 or len(yshp) != 3:  # [party, M, K] . [party, K, N] only
            return None
        m, nout = shp[1], yshp[2]
        if m * nout < (1 << 20):
            return None
        bits = x0.v.bits
        nonce = self.nonce(plc)
        main = torch.cuda.current_stream(self.device)
        side = getattr(self, "_side_stream", None)
        if side is None:
            side = self._side_stream = torch.cuda.Stream(self.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            r = R.prf_expand_k(self.key_ptr(plc, 0), 3, nonce, (m, nout), bits, self.device)
        v = R.dot_cross(x0.v, x1.v, y0.v, y1.v, nb=1)
        main.wait_stream(side)
        r.data.record_stream(main)
        s0, s1 = R.add_zs3(v, r)
        self.stats.record_round(_nbytes(s0))
        return PV(plc, s0), PV(plc, s1)

    def p_prepare_cross(self, plc, y0, y1):
        """The B' operand of p_dot_cross, limb-split once for several row blocks."""
        return R.PreparedCross(y0.v, y1.v)

    # every party of a session on this device: a pair's second share vector is its first
    # rolled by one party (s1[p] = s0[p + 1]), so the CRT GEMM needs the residues of s0 only
    pair_rolled = os.environ.get("MOOSEX_PAIR_ROLL", "1") != "0"
    # products with every dimension >= 256 take the asymmetric local products
    # (ops/ring.py dot_cross_asym) on every device, so CPU and GPU sessions agree bitwise
    dot_asym = os.environ.get("MOOSEX_DOT_ASYM", "1") != "0"

    def p_dot_cross_rows(self, plc, x0, x1, r0, r1, prepared):
        if self.pair_rolled:
            v = R.dot_cross_pair(x0.v, None, None, 1, pb=prepared, r0=r0, r1=r1)
            if v is not None:
                return PV(plc, v)
        return PV(plc, R.dot_cross_rows(x0.v, x1.v, r0, r1, prepared))

    def p_dot_cross(self, plc, x0, x1, y0, y1, nbatch=0):
        """``nbatch`` leading logical axes are batch axes (independent products, one
        batched GEMM launch with the parties).  A right operand used by several products of
        one evaluation (e.g. a chain z = z.y) has its GEMM operand image prepared once, from
        its second use on; every product is still computed."""
        yv0, yv1 = y0.v, y1.v
        if nbatch == 0 and self.dot_asym and _asym_applies(x0.v, yv0):
            # the asymmetric local products (five K-long GEMMs instead of six; same sum)
            return PV(plc, R.dot_cross_asym(x0.v, x1.v, yv0, yv1, rolled=self.pair_rolled))
        # (not while dataflow lanes run: a prepared image produced on one lane would be
        # read by products on other lanes without an event)
        if (nbatch == 0 and self.device.type == "cuda" and len(yv0.shape) == 3
                and not _lanes.ACTIVE
                and len(x0.v.shape) == 3 and min(x0.v.shape[1], yv0.shape[1], yv0.shape[2]) >= 256):
            # (large products only: small ones run the VALU GEMM, which has no prepared form)
            cache = self.__dict__.setdefault("_prepared_b", {})
            key = (id(yv0.data), id(yv1.data))
            hit = cache.get(key)
            if hit is not None and hit[0] is yv0.data and hit[1] is yv1.data:
                pb = hit[2]
                if pb is None:  # second use: prepare once for this and every later product
                    pb = R.PreparedCross(yv0, yv1)
                    cache[key] = (yv0.data, yv1.data, pb)
                if pb.lb is not None:
                    return self.p_dot_cross_rows(plc, x0, x1, 0, x0.v.shape[1], pb)
            elif len(cache) < 64:
                cache[key] = (yv0.data, yv1.data, None)  # holds the tensors: ids stay unique
        if (nbatch == 0 and self.pair_rolled and self.device.type == "cuda"
                and len(yv0.shape) == 3):
            v = R.dot_cross_pair(x0.v, yv0, yv1, 1)
            if v is not None:
                return PV(plc, v)
        return PV(plc, R.dot_cross(x0.v, x1.v, y0.v, y1.v, nb=1 + nbatch))

    def end_evaluation(self, ok=True):
        """Drop per-evaluation caches (prepared GEMM operands hold device memory and must
        not outlive the evaluation whose values they were prepared from)."""
        self.__dict__.pop("_prepared_b", None)

    def p_add_zero_share(self, plc, z, kind="arith"):
        return PV(plc, R.rss_cross_k(kind, z.v, None, None, None, self.key_ptr(plc, 0), 3,
                                     self.nonce(plc), 3))

    def p_shape(self, x: PV):
        return tuple(x.v.shape[1:])

    # -- fused whole-protocol kernels (same shares as the generic protocol code) ------
    fused = os.environ.get("MOOSEX_FUSED", "1") != "0"

    def fused_trunc_pr_premul(self, x, m, nonces, c: int):
        """fused_trunc_pr of c * x for a public integer c (mul_public folded into the
        TruncPr kernel; c is a host value, so nothing is read back from the device)."""
        import ctypes

        from moose_amd.ops import native as nat

        s0 = x.s0.v.data.contiguous()
        n = x.s0.v.numel() // 3
        nn = (ctypes.c_uint64 * 6)(*[v & ((1 << 64) - 1) for v in nonces])
        cv = int(c) % (1 << x.bits)
        cm = (ctypes.c_uint64 * 2)(cv & ((1 << 64) - 1), cv >> 64)
        out0, out1 = (t.data for t in R.ring4(x.s0.v.shape, x.bits, s0.device))
        nat.check(nat.lib().mx_trunc_pr3_kmo(
            nat.dev_of(s0), R._words(x.bits), nat.ptr(s0), nat.ptr(out0), nat.ptr(out1), n, m,
            self.key_ptr(x.plc, 0), self.key_ptr(x.plc, 2), nn, n, cm, nat.stream_of(s0)),
            "trunc_pr3 (premultiplied)")
        self._trunc_traffic(x, out0.numel() * out0.element_size() // 3)
        return PV(x.plc, R.RT(out0, x.bits)), PV(x.plc, R.RT(out1, x.bits))

    def fused_trunc_pr(self, x, m, nonces, out=None):
        """All three parties' TruncPr in one kernel (see replicated.trunc_pr).  ``out``:
        optional (s0, s1) party-vector views (each party's slot dense, e.g. rows of a larger
        stack) that the kernel writes in place."""
        import ctypes

        from moose_amd.ops import native as nat

        s0 = x.s0.v.data.contiguous()
        n = x.s0.v.numel() // 3
        nn = (ctypes.c_uint64 * 6)(*[v & ((1 << 64) - 1) for v in nonces])
        keys = (self.key_ptr(x.plc, 0), self.key_ptr(x.plc, 2))
        if out is not None:
            out0, out1 = out[0].v.data, out[1].v.data
            w = 2 if x.bits == 128 else 1  # int64 words per element
            os_ = out0.stride(0)
            if not (out0.shape == s0.shape and out1.shape == s0.shape
                    and out1.stride(0) == os_ and out0[0].is_contiguous()
                    and out1[0].is_contiguous() and os_ % w == 0 and os_ // w >= n):
                raise ValueError("fused_trunc_pr: out views must hold dense party slots")
            os_ //= w
            nat.check(nat.lib().mx_trunc_pr3_ko(
                nat.dev_of(s0), R._words(x.bits), nat.ptr(s0), nat.ptr(out0), nat.ptr(out1), n, m,
                *keys, nn, os_, nat.stream_of(s0)), "trunc_pr3 (views)")
            self._trunc_traffic(x, out0[0].numel() * out0.element_size())
            return out[0], out[1]
        out0, out1 = (t.data for t in R.ring4(x.s0.v.shape, x.bits, s0.device))
        nat.check(
            nat.lib().mx_trunc_pr3_k(
                nat.dev_of(s0), R._words(x.bits), nat.ptr(s0), nat.ptr(out0), nat.ptr(out1), n, m,
                *keys, nn, nat.stream_of(s0),
            ),
            "trunc_pr3",
        )
        self._trunc_traffic(x, out0.numel() * out0.element_size() // 3)
        return PV(x.plc, R.RT(out0, x.bits)), PV(x.plc, R.RT(out1, x.bits))

    def p_wsum_trunc_add(self, plc, S, weights, m, cadd: int):
        """rep.trunc_pr(weighted sum of the powers stack ``S`` (a party vector [3, R, ...]),
        m) + the public constant ``cadd`` on party 0's share, in one launch
        (k_wsum_trunc3_lat); the nonces drawn as trunc_pr draws them.  None -> the three
        steps."""
        import ctypes

        from moose_amd.ops import native as nat

        v = S.v
        if (self.device.type != "cuda" or not isinstance(v, R.RT) or v.bits not in (64, 128)
                or not m or len(v.shape) < 2):
            return None
        d = v.data
        w = 2 if v.bits == 128 else 1
        Rr, inner = v.shape[1], math.prod(v.shape[2:])
        if (d.stride(0) % w or d.stride(1) % w or not d[0, 0].is_contiguous()
                or d[0, 0].numel() != inner * w or Rr != len(weights)):
            return None
        nblk = inner if w == 2 else (inner + 1) // 2
        if inner == 0 or nblk > 8192:
            return None
        wt = R.const_ints([int(x) % (1 << v.bits) for x in weights], v.bits, self.device)
        nr0, nr1, nt, nm, n0, n2 = (self.nonce(plc) for _ in range(6))
        nn = (ctypes.c_uint64 * 6)(*[x & ((1 << 64) - 1) for x in (nr0, nr1, nt, nm, n0, n2)])
        c = cadd % (1 << v.bits)
        ca = (ctypes.c_uint64 * 2)(c & ((1 << 64) - 1), c >> 64)
        out0, out1 = (t.data for t in R.ring4((3,) + tuple(v.shape[2:]), v.bits, d.device))
        nat.check(nat.lib().mxh_wsum_trunc3(
            R._words(v.bits), nat.ptr(d), d.stride(0) // w, d.stride(1) // w, Rr,
            nat.ptr(wt.data), nat.ptr(out0), nat.ptr(out1), inner, int(m),
            ctypes.c_void_p(self.key_ptr(plc, 0)), ctypes.c_void_p(self.key_ptr(plc, 2)), nn, ca,
            nat.stream_of(d)), "wsum_trunc3")
        x = type("X", (), {})()
        x.plc = plc
        self._trunc_traffic(x, out0.numel() * out0.element_size() // 3)
        return PV(plc, R.RT(out0, v.bits)), PV(plc, R.RT(out1, v.bits))

    def _trunc_traffic(self, x, nbytes):
        o = x.plc.owners
        # messages of the protocol: dealer -> P1 (2 tensors), P0 <-> P1 (two rounds)
        st = self.stats
        for src, dst in ((o[2], o[1]), (o[0], o[1]), (o[1], o[0])):
            st.record_send(src, dst, nbytes, count=2)
        st.record_round(2 * nbytes, count=2)

    def fused_share(self, plc, x: HV, j, kind, n1, na):
        import ctypes

        from moose_amd.ops import native as nat

        code, xd, aux = R.share_source(x.v, kind)  # a pending encoding: encoded in-kernel
        d = self.share_dir(plc, j)
        out0, out1 = (t.data for t in R.ring4((3,) + tuple(x.v.shape), x.v.bits, xd.device))
        nat.check(
            nat.lib().mx_share3_k(
                nat.dev_of(xd), code | (R.SHARE_MIRROR if d == 2 else 0), R._words(x.v.bits),
                nat.ptr(xd), nat.ptr(out0), nat.ptr(out1), x.v.numel(), j,
                ctypes.c_void_p(self.key_ptr(plc, (j + d - 1) % 3)),
                ctypes.c_void_p(self.key_ptr(plc, 3)), n1, na if aux is None else aux,
                nat.stream_of(xd),
            ),
            "share3",
        )
        self.stats.record_send(x.host, plc.owners[(j + d) % 3], _nbytes(x.v))
        return PV(plc, R.RT(out0, x.v.bits)), PV(plc, R.RT(out1, x.v.bits))

    def mirror(self, x: HV, plc):
        """Host value -> mirrored (public on the 3 hosts of ``plc``)."""
        from moose_amd.runtime.values import MV

        for o in plc.owners:
            if o != x.host:
                self.stats.record_send(x.host, o, _nbytes(x.v))
        return MV(plc, x.v)

    def materialized(self, x) -> bool:
        return True


def _stack3(v):
    if isinstance(v, R.RT):
        return R.RT(v.data.unsqueeze(0).expand((3,) + tuple(v.data.shape)).contiguous(), v.bits)
    return v.unsqueeze(0).expand((3,) + tuple(v.shape)).contiguous()
