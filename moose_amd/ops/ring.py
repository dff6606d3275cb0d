"""Ring tensors: Z_2^64, Z_2^128 and Z_2 (bits) on CPU or MI355X.

``RT`` wraps a torch tensor:

* Z_2^64  -> ``torch.int64`` of the logical shape (two's complement = u64 bits),
* Z_2^128 -> ``torch.int64`` of shape ``(*shape, 2)`` holding (lo, hi) words, i.e. the
  in-memory layout of ``unsigned __int128``; the native kernels read it as such,
* Z_2     -> ``torch.uint8`` holding 0/1.

Elementwise Z_2^64 / Z_2 arithmetic uses torch's wrapping integer kernels; everything
that torch cannot express (Z_2^128 arithmetic, exact ring GEMM, AES-CTR PRG, the fused RSS
step) goes to ``libmoosex`` (``csrc/``), on the tensor's device and current HIP stream.

Axis arguments are *logical*: ``nb`` leading batch dimensions (e.g. the party axis of a
stacked 3-party session) are skipped.

Parity: reference host ring kernels ``moose/src/host/ops.rs:1709-2036``.
"""
from __future__ import annotations

import builtins
import ctypes
import math
import os
import threading
from typing import List
from typing import Sequence

import numpy as np
import torch

from moose_amd.ops import native as nat

MASK64 = (1 << 64) - 1
MASK128 = (1 << 128) - 1

_BIN = {"add": 0, "sub": 1, "mul": 2, "and": 3, "or": 4, "xor": 5}
_UN = {"neg": 0, "not": 1, "shl": 2, "shr": 3, "sar": 4}
_CMP = {"lt": 0, "gt": 1, "eq": 2, "msb": 3}


# Every host->device copy made while a computation runs goes through to_device, so that
# hipGraph capture (runtime/graphs.py) can substitute copies staged before the capture.
# The hook is per thread (in-process parties record and capture on their own threads).
_UPLOAD_HOOK = None  # process-wide fallback
_TLS = threading.local()


def upload_hook():
    h = getattr(_TLS, "hook", None)
    return h if h is not None else _UPLOAD_HOOK


def set_upload_hook(hook):
    """Install ``hook`` for the calling thread; returns the previous one."""
    prev = getattr(_TLS, "hook", None)
    _TLS.hook = hook
    return prev


def to_device(t: torch.Tensor, device) -> torch.Tensor:
    device = torch.device(device)
    if device.type == "cpu" or t.device == device:
        return t
    hook = upload_hook()
    if hook is not None:
        return hook(t, device)
    return t.to(device)


def _words(bits):
    return {1: 0, 64: 1, 128: 2}[bits]


class RT:
    """A ring tensor (see module docstring)."""

    __slots__ = ("data", "bits", "_shape")

    def __init__(self, data: torch.Tensor, bits: int):
        self.data = data
        self.bits = bits
        self._shape = None

    # -- shape -------------------------------------------------------------
    @property
    def shape(self):
        s = self._shape
        if s is None:  # computed once: shapes are read several times per launch
            s = tuple(self.data.shape)
            s = self._shape = s[:-1] if self.bits == 128 else s
        return s

    @property
    def ndim(self):
        return len(self.shape)

    @property
    def device(self):
        return self.data.device

    def numel(self):
        return math.prod(self.shape)

    def __repr__(self):
        return f"RT(bits={self.bits}, shape={self.shape}, device={self.device})"

    def contiguous(self):
        return RT(self.data.contiguous(), self.bits)

    def clone(self):
        return RT(self.data.clone(), self.bits)

    # -- arithmetic --------------------------------------------------------
    def __add__(self, o):
        return binary("add", self, o)

    def __sub__(self, o):
        return binary("sub", self, o)

    def __mul__(self, o):
        return binary("mul", self, o)

    def __and__(self, o):
        return binary("and", self, o)

    def __or__(self, o):
        return binary("or", self, o)

    def __xor__(self, o):
        return binary("xor", self, o)

    def __neg__(self):
        return unary("neg", self)

    def __invert__(self):
        return unary("not", self)

    def shl(self, k):
        return unary("shl", self, k)

    def shr(self, k):
        return unary("shr", self, k)

    def sar(self, k):
        return unary("sar", self, k)


# ---------------------------------------------------------------------------
# construction / conversion
# ---------------------------------------------------------------------------
def empty(shape, bits, device) -> RT:
    shape = tuple(shape)
    if bits == 128:
        return RT(torch.empty(shape + (2,), dtype=torch.int64, device=device), 128)
    if bits == 64:
        return RT(torch.empty(shape, dtype=torch.int64, device=device), 64)
    return RT(torch.empty(shape, dtype=torch.uint8, device=device), 1)


def empty2(shape, bits, device):
    """Two ring tensors of one shape from ONE allocation (the paired outputs of the share-
    pair / stacked-protocol kernels)."""
    both = empty((2,) + tuple(shape), bits, device).data
    return RT(both[0], bits), RT(both[1], bits)


_RING4 = os.environ.get("MOOSEX_RING4", "1") != "0"


def ring4(shape, bits, device):
    """The two share vectors of a stacked replicated value ([3, ...]) as views of ONE
    [4, ...] buffer holding slots x0, x1, x2, x0: s0 = buf[0:3], s1 = buf[1:4] = s0 rolled
    by one party.  Pair-producing kernels detect out1 == out0 + slot and write 4 slots, not
    6; every consumer sees two ordinary contiguous [3, ...] tensors."""
    shape = tuple(shape)
    if not shape or shape[0] != 3 or not _RING4:
        return empty2(shape, bits, device)
    buf = empty((4,) + shape[1:], bits, device).data
    return RT(buf[0:3], bits), RT(buf[1:4], bits)


def zeros(shape, bits, device) -> RT:
    r = empty(shape, bits, device)
    r.data.zero_()
    return r


_SCALARS = {}
# > 0 while several threads issue work on their own streams of one device (the in-process
# parties, parallel/threads.py): a cached constant is then read by other streams too.  A
# count, so that overlapping evaluations of several runtimes do not clear it for each other
SHARED_STREAMS = 0
_SHARED_LOCK = threading.Lock()


def shared_streams(delta: int):
    global SHARED_STREAMS
    with _SHARED_LOCK:
        SHARED_STREAMS = max(0, SHARED_STREAMS + delta)


# MOOSEX_CONST_CACHE=0: no shared device constants (every use makes its own; diagnostics)
CONST_CACHE = os.environ.get("MOOSEX_CONST_CACHE", "1") != "0"


def _cache_put(cache, key, t, limit):
    """Insert a freshly made device constant into a shared cache.  While dataflow lanes
    run (runtime/lanes.py) other streams may read it next, so the producing stream is
    drained first (once per constant)."""
    if len(cache) >= limit or not CONST_CACHE:
        return
    from moose_amd.runtime import lanes

    d = t[1].data if isinstance(t, tuple) else t.data
    if (lanes.ACTIVE or SHARED_STREAMS) and d.is_cuda:
        torch.cuda.current_stream(d.device).synchronize()
    with _SHARED_LOCK:
        # first in wins: parties on threads may make one constant at once, and an entry
        # keyed by an object's id must keep that object alive (never replaced)
        cache.setdefault(key, t)


def fill(shape, value: int, bits, device) -> RT:
    """Constant ring tensor (``value`` taken mod 2^bits).

    Scalars (shape ``()``) are the public constants of the protocols (encoded
    coefficients, masks, 1/n ...); they are created once per device and shared -- callers
    never write into a fill result.  Not while a hipGraph is being captured: the tensor
    would live in the graph's private pool."""
    shape = tuple(shape)
    if not shape:
        key = (int(value), bits, str(device))
        hit = _SCALARS.get(key)
        if hit is not None:
            return hit
        t = _fill(shape, value, bits, device)
        if torch.device(device).type == "cpu" or not torch.cuda.is_current_stream_capturing():
            _cache_put(_SCALARS, key, t, 65536)
        return t
    return _fill(shape, value, bits, device)


def _fill(shape, value: int, bits, device) -> RT:
    if bits == 1:
        return RT(torch.full(shape, int(value) & 1, dtype=torch.uint8, device=device), 1)
    if bits == 64:
        v = _to_i64(int(value) & MASK64)
        return RT(torch.full(shape, v, dtype=torch.int64, device=device), 64)
    v = int(value) & MASK128
    lo, hi = _to_i64(v & MASK64), _to_i64(v >> 64)
    # one native fill kernel (slice assignment of a python int would be a host->device
    # copy, which is not allowed while a hipGraph is being captured)
    out = empty(shape, 128, device)
    nat.check(nat.lib().mx_fill(nat.dev_of(out.data), 2, nat.ptr(out.data), math.prod(shape),
                                lo & MASK64, hi & MASK64, nat.stream_of(out.data)), "fill")
    return out


def _to_i64(u):
    u &= MASK64
    return u - (1 << 64) if u >= (1 << 63) else u


def from_ints(values, bits, device="cpu") -> RT:
    """Build from python ints / nested lists (values reduced mod 2^bits)."""
    arr = np.array(values, dtype=object)
    shape = arr.shape
    flat = [int(x) for x in arr.reshape(-1)]
    if bits == 1:
        t = torch.tensor([v & 1 for v in flat], dtype=torch.uint8).reshape(shape)
        return RT(to_device(t, device), 1)
    if bits == 64:
        t = torch.tensor([_to_i64(v) for v in flat], dtype=torch.int64).reshape(shape)
        return RT(to_device(t, device), 64)
    pairs = [[_to_i64(v & MASK64), _to_i64((v >> 64) & MASK64)] for v in flat]
    t = torch.tensor(pairs, dtype=torch.int64).reshape(shape + (2,))
    return RT(to_device(t, device), 128)


def to_ints(x: RT) -> np.ndarray:
    """Unsigned python-int view (object ndarray) -- test/inspection helper."""
    d = x.data.detach().cpu()
    if x.bits == 1:
        return d.numpy().astype(object)
    if x.bits == 64:
        return np.vectorize(lambda v: int(v) & MASK64, otypes=[object])(d.numpy())
    a = d.numpy()
    lo = np.vectorize(lambda v: int(v) & MASK64, otypes=[object])(a[..., 0])
    hi = np.vectorize(lambda v: int(v) & MASK64, otypes=[object])(a[..., 1])
    return lo + hi * (1 << 64)


def to_signed_ints(x: RT) -> np.ndarray:
    u = to_ints(x)
    half = 1 << (x.bits - 1)
    return np.vectorize(lambda v: v - (1 << x.bits) if v >= half else v, otypes=[object])(u)


# ---------------------------------------------------------------------------
# elementwise
# ---------------------------------------------------------------------------
def _as_rt(o, like: RT) -> RT:
    if isinstance(o, RT):
        return o
    if isinstance(o, int):
        return fill((), o, like.bits, like.device)
    raise TypeError(f"cannot combine RT with {type(o)}")


def _broadcast(a: RT, b: RT):
    if a.shape == b.shape:
        return a, b
    shp = torch.broadcast_shapes(a.shape, b.shape)
    return expand(a, shp), expand(b, shp)


def expand(a: RT, shape) -> RT:
    shape = tuple(shape)
    if a.shape == shape:
        return a
    if a.bits == 128:
        return RT(a.data.expand(shape + (2,)), 128)
    return RT(a.data.expand(shape), a.bits)


def binary(op: str, a, b, alloc=None) -> RT:
    """a op b elementwise; ``alloc(shape, dtype)``: where the result goes (a session's
    outbox when it is a message; Z_2^64 / Z_2^128 only)."""
    if not isinstance(a, RT):
        a = _as_rt(a, b)
    b = _as_rt(b, a)
    if a.bits != b.bits:
        raise TypeError(f"ring width mismatch {a.bits} vs {b.bits}")
    bits = a.bits
    if bits == 1:
        x, y = a.data, b.data
        if op in ("add", "sub", "xor"):
            return RT(x ^ y, 1)
        if op in ("mul", "and"):
            return RT(x & y, 1)
        if op == "or":
            return RT(x | y, 1)
    # Z_2^64 / Z_2^128: one native kernel (libmoosex, gfx950 on the device); scalar
    # operands broadcast natively, other broadcasts are expanded first
    na, nb_ = a.numel(), b.numel()
    if na != nb_ and na != 1 and nb_ != 1:
        a, b = _broadcast(a, b)
        na = nb_ = a.numel()
    n = max(na, nb_)
    out_shape = a.shape if na >= nb_ else b.shape
    out = _empty_in(alloc, out_shape, bits, a.device)
    ad, bd = a.data.contiguous(), b.data.contiguous()
    nat.check(
        nat.lib().mx_ew_binary(
            nat.dev_of(ad), _BIN[op], _words(bits), nat.ptr(ad), na, nat.ptr(bd), nb_,
            nat.ptr(out.data), n, nat.stream_of(ad),
        ),
        f"ring{bits} {op}",
    )
    return out


def unary(op: str, a: RT, k: int = 0) -> RT:
    bits = a.bits
    if bits == 1:
        if op == "neg":
            return RT(a.data.clone(), 1)
        if op == "not":
            return RT(a.data ^ 1, 1)
        return RT(a.data.clone() if k == 0 else torch.zeros_like(a.data), 1)
    out = empty(a.shape, bits, a.device)
    ad = a.data.contiguous()
    nat.check(
        nat.lib().mx_ew_unary(
            nat.dev_of(ad), _UN[op], _words(bits), nat.ptr(ad), nat.ptr(out.data), a.numel(),
            int(k), nat.stream_of(ad),
        ),
        f"ring128 {op}",
    )
    return out


def transpose2(a0: RT, a1: RT):
    """(a0^T, a1^T) of two [rows, cols] ring matrices (a party's share components) in one
    launch (mx_transpose2: 32 x 32 tiles through LDS) instead of two strided copies."""
    rows, cols = a0.shape
    bits = a0.bits
    d0, d1 = a0.data.contiguous(), a1.data.contiguous()
    o0, o1 = empty2((cols, rows), bits, d0.device)
    nat.check(nat.lib().mx_transpose2(
        nat.dev_of(d0), _words(bits), nat.ptr(d0), nat.ptr(o0.data), nat.ptr(d1),
        nat.ptr(o1.data), rows, cols, nat.stream_of(d0)), "transpose2")
    return o0, o1


def binary2(op: str, a0: RT, b0: RT, a1: RT, b1: RT):
    """(a0 op b0, a1 op b1) -- both share vectors of a share-wise replicated op -- in one
    launch (mx_ew_binary2).  Operands of each pair have the same shapes as the other pair's;
    anything else (bit tensors, general broadcasts) takes two binary() calls."""
    bits = a0.bits
    na, nb_ = a0.numel(), b0.numel()
    if (bits == 1 or not all(isinstance(t, RT) and t.bits == bits for t in (b0, a1, b1))
            or a1.shape != a0.shape or b1.shape != b0.shape
            or (na != nb_ and na != 1 and nb_ != 1)):
        return binary(op, a0, b0), binary(op, a1, b1)
    n = max(na, nb_)
    shp = a0.shape if na >= nb_ else b0.shape
    o0, o1 = empty2(shp, bits, a0.device)
    d = [t.data.contiguous() for t in (a0, b0, a1, b1)]
    nat.check(nat.lib().mx_ew_binary2(
        nat.dev_of(d[0]), _BIN[op], _words(bits), nat.ptr(d[0]), nat.ptr(d[1]),
        nat.ptr(o0.data), nat.ptr(d[2]), nat.ptr(d[3]), nat.ptr(o1.data), na, nb_, n,
        nat.stream_of(d[0])), f"ring{bits} {op} (pair)")
    return o0, o1


def unary2(op: str, a0: RT, a1: RT, k: int = 0):
    """(op a0, op a1) in one launch (mx_ew_unary2)."""
    if a0.bits == 1 or a1.bits != a0.bits or a1.shape != a0.shape:
        return unary(op, a0, k), unary(op, a1, k)
    o0, o1 = empty2(a0.shape, a0.bits, a0.device)
    d0, d1 = a0.data.contiguous(), a1.data.contiguous()
    nat.check(nat.lib().mx_ew_unary2(
        nat.dev_of(d0), _UN[op], _words(a0.bits), nat.ptr(d0), nat.ptr(o0.data), nat.ptr(d1),
        nat.ptr(o1.data), a0.numel(), int(k), nat.stream_of(d0)), f"ring{a0.bits} {op} (pair)")
    return o0, o1


def compare(op: str, a: RT, b: RT = None) -> RT:
    """Signed comparison -> bit tensor (op: lt, gt, eq, msb)."""
    if a.bits == 64 and op != "msb":
        x, y = a.data, b.data
        r = {"lt": x < y, "gt": x > y, "eq": x == y}[op]
        return RT(r.to(torch.uint8), 1)
    if a.bits == 64:
        return RT(((a.data >> 63) & 1).to(torch.uint8), 1)
    if b is not None and a.shape != b.shape and b.numel() != 1 and a.numel() != 1:
        a, b = _broadcast(a, b)
    n = max(a.numel(), b.numel() if b is not None else 0)
    shape = a.shape if b is None or a.numel() >= b.numel() else b.shape
    out = torch.empty(shape, dtype=torch.uint8, device=a.device)
    ad = a.data.contiguous()
    bd = b.data.contiguous() if b is not None else None
    nat.check(
        nat.lib().mx_ew_compare(
            nat.dev_of(ad), _CMP[op], _words(a.bits), nat.ptr(ad), a.numel(), nat.ptr(bd),
            b.numel() if b is not None else 0, nat.ptr(out), n, nat.stream_of(ad),
        ),
        f"compare {op}",
    )
    return RT(out, 1)


def bit_extract(a: RT, bit: int) -> RT:
    if a.data.is_cuda and a.bits in (64, 128) and 0 <= bit < a.bits:  # one kernel
        ad = a.data.contiguous()
        out = torch.empty(a.shape, dtype=torch.uint8, device=ad.device)
        nat.check(nat.lib().mx_bit_extract(nat.dev_of(ad), _words(a.bits), nat.ptr(ad),
                                           nat.ptr(out), out.numel(), bit, nat.stream_of(ad)),
                  "bit_extract")
        return RT(out, 1)
    if a.bits == 64:
        return RT(((a.data >> bit) & 1).to(torch.uint8), 1)
    w = a.data[..., bit // 64]
    return RT(((w >> (bit % 64)) & 1).to(torch.uint8), 1)


def ring_inject(bitsrt: RT, bit: int, ring_bits: int) -> RT:
    """bit tensor -> ring tensor with the bit placed at position ``bit``."""
    if bitsrt.data.is_cuda and ring_bits in (64, 128) and 0 <= bit < ring_bits:  # one kernel
        bd = bitsrt.data.contiguous()
        if bd.dtype != torch.uint8:
            bd = bd.to(torch.uint8)
        out = empty(tuple(bd.shape), ring_bits, bd.device)
        nat.check(nat.lib().mx_ring_inject(nat.dev_of(bd), _words(ring_bits), nat.ptr(bd),
                                           nat.ptr(out.data), bd.numel(), bit,
                                           nat.stream_of(bd)), "ring_inject")
        return out
    b = bitsrt.data.to(torch.int64) & 1
    if ring_bits == 64:
        return RT(b << bit if bit < 64 else torch.zeros_like(b), 64)
    out = torch.zeros(tuple(b.shape) + (2,), dtype=torch.int64, device=b.device)
    if bit < 64:
        out[..., 0] = b << bit
    else:
        out[..., 1] = b << (bit - 64)
    return RT(out, 128)


def cast(a: RT, bits: int) -> RT:
    """Ring width change: truncation 128->64, zero extension 64->128, bit->ring."""
    if a.bits == bits:
        return a
    if a.bits == 128 and bits == 64:
        return RT(a.data[..., 0].contiguous(), 64)
    if a.bits == 64 and bits == 128:
        out = torch.zeros(tuple(a.data.shape) + (2,), dtype=torch.int64, device=a.device)
        out[..., 0] = a.data
        return RT(out, 128)
    if a.bits == 1:
        return ring_inject(a, 0, bits)
    if bits == 1:
        return bit_extract(a, 0)
    raise TypeError(f"cannot cast ring {a.bits} -> {bits}")


def sign_extend(a: RT, from_bits: int, bits: int) -> RT:
    """64 -> 128 with sign extension."""
    assert a.bits == 64 and bits == 128
    out = torch.empty(tuple(a.data.shape) + (2,), dtype=torch.int64, device=a.device)
    out[..., 0] = a.data
    out[..., 1] = a.data >> 63
    return RT(out, 128)


# ---------------------------------------------------------------------------
# fixed-point encode / decode (reference host/fixedpoint.rs: truncating `as i128`)
# ---------------------------------------------------------------------------
def encode(x: torch.Tensor, frac: int, bits: int) -> RT:
    x = x.to(torch.float64).contiguous()
    out = empty(tuple(x.shape), bits, x.device)
    nat.check(
        nat.lib().mx_encode(
            nat.dev_of(x), _words(bits), nat.ptr(x), nat.ptr(out.data), x.numel(), int(frac),
            nat.stream_of(x),
        ),
        "encode",
    )
    return out


def _stream_of(t: torch.Tensor):
    """The current stream of ``t``'s device (None on the host): where a lazy value's inputs
    were issued."""
    return torch.cuda.current_stream(t.device) if t.is_cuda else None


def _join(stream):
    """Order the current stream after the work issued so far on ``stream`` -- a lazy value
    created on one stream and consumed on another (dataflow lanes, step streams)."""
    if stream is not None:
        cur = torch.cuda.current_stream(stream.device)
        if cur != stream:
            cur.wait_stream(stream)


class Encoded(RT):
    """A float64 tensor's fixed-point encoding (x * 2^frac), formed on first use of
    ``data``.  Input sharing of it encodes inside the share kernel (kind MX_SHARE_F64): the
    ring-valued encoding never goes to memory."""

    __slots__ = ("src", "frac", "stream")

    def __init__(self, x: torch.Tensor, frac: int, bits: int):
        _RT_DATA.__set__(self, None)
        self.bits = bits
        self._shape = tuple(x.shape)
        self.src = x
        self.frac = int(frac)
        self.stream = _stream_of(x)

    def pending(self) -> bool:
        return _RT_DATA.__get__(self) is None

    @property
    def data(self):
        d = _RT_DATA.__get__(self)
        if d is None:
            _join(self.stream)
            d = encode(self.src, self.frac, self.bits).data
            _RT_DATA.__set__(self, d)
            self.src = None
        return d

    @data.setter
    def data(self, v):
        _RT_DATA.__set__(self, v)

    @property
    def device(self):
        return self.src.device if self.pending() else self.data.device


# ids of cached computation constants (runtime/interpreter.py _CONST_LV keeps them alive)
CONST_IDS = set()
_ENCODED_CONSTS = {}


def encode_lazy(x: torch.Tensor, frac: int, bits: int) -> RT:
    """encode(), deferred to the first use (:class:`Encoded`) for 64/128-bit rings; a
    cached computation constant is encoded once (not while a hipGraph is being captured:
    the result would live in the graph's pool)."""
    if id(x) in CONST_IDS and x.is_cuda:
        key = (id(x), int(frac), bits)
        hit = _ENCODED_CONSTS.get(key)
        # the entry holds its source tensor: an id is only ever matched while that very
        # tensor lives (a freed tensor's id may come back as another tensor's)
        if hit is not None and hit[0] is x:
            return hit[1]
        if not torch.cuda.is_current_stream_capturing():
            e = encode(x, frac, bits)
            _cache_put(_ENCODED_CONSTS, key, (x, e), 4096)
            return e
    if bits not in (64, 128):
        return encode(x, frac, bits)
    return Encoded(x.to(torch.float64).contiguous(), frac, bits)


def share_source(x: RT, kind: str):
    """(kind code, device tensor, aux) for the share kernels: an unencoded float64 input is
    passed as is (MX_SHARE_F64 = 2, aux = its fractional bits), else the ring data."""
    if kind == "arith" and isinstance(x, Encoded) and x.pending():
        _join(x.stream)
        return 2, x.src, x.frac
    return (1 if kind == "bool" else 0), x.data.contiguous(), None


def decode(a: RT, frac: int) -> torch.Tensor:
    if isinstance(a, Opened) and a.pending():  # the reveal's add fused into the decode
        _join(a.stream)
        d = [t.data.contiguous() for t in a.parts]
        out = torch.empty(a.shape, dtype=torch.float64, device=a.device)
        ptrs = [nat.ptr(x) for x in d] + [None] * (4 - len(d))
        nat.check(nat.lib().mx_addn_decode(
            nat.dev_of(d[0]), _words(a.bits), *ptrs, nat.ptr(out), a.numel(),
            int(frac), nat.stream_of(d[0])), "addn_decode")
        return out
    ad = a.data.contiguous()
    out = torch.empty(a.shape, dtype=torch.float64, device=a.device)
    nat.check(
        nat.lib().mx_decode(
            nat.dev_of(ad), _words(a.bits), nat.ptr(ad), nat.ptr(out), a.numel(), int(frac),
            nat.stream_of(ad),
        ),
        "decode",
    )
    return out


# ---------------------------------------------------------------------------
# shape ops (logical axes after `nb` batch dims)
# ---------------------------------------------------------------------------
def _ax(a: RT, axis: int, nb: int) -> int:
    nd = a.ndim - nb
    if axis < 0:
        axis += nd
    if not 0 <= axis < max(nd, 1):
        raise IndexError(f"axis {axis} out of range for logical rank {nd}")
    return axis + nb


def reshape(a: RT, shape, nb=0) -> RT:
    shape = tuple(int(s) for s in shape)
    full = a.shape[:nb] + shape
    if a.bits == 128:
        return RT(a.data.reshape(full + (2,)), 128)
    return RT(a.data.reshape(full), a.bits)


def transpose(a: RT, nb=0, perm=None) -> RT:
    nd = a.ndim - nb
    perm = list(range(nd))[::-1] if perm is None else list(perm)
    full = list(range(nb)) + [p + nb for p in perm]
    if a.bits == 128:
        full.append(a.ndim)
    return RT(a.data.permute(full).contiguous(), a.bits)


def expand_dims(a: RT, axes, nb=0) -> RT:
    d = a.data
    nd = a.ndim - nb
    for ax in sorted(int(x) for x in axes):
        if ax < 0:
            ax += nd + 1
        d = d.unsqueeze(ax + nb)
        nd += 1
    return RT(d, a.bits)


def squeeze(a: RT, axis=None, nb=0) -> RT:
    if axis is None:
        shape = a.shape[:nb] + tuple(s for s in a.shape[nb:] if s != 1)
        return reshape(a, shape[nb:], nb)
    ax = _ax(a, axis, nb)
    return RT(a.data.squeeze(ax), a.bits)


def concat(xs: Sequence[RT], axis=0, nb=0) -> RT:
    ax = _ax(xs[0], axis, nb)
    return RT(torch.cat([x.data for x in xs], dim=ax), xs[0].bits)


def index_axis(a: RT, axis: int, index: int, nb=0) -> RT:
    ax = _ax(a, axis, nb)
    v = a.data.select(ax, index)
    if nb == 1 and ax == 1 and v.dim() >= 1 and v[0].is_contiguous():
        # one entry of a party-stacked batch ([P, k, ...] -> [P, ...]): a view whose party
        # slots stay dense -- consumers read it in place or copy on demand
        return RT(v, a.bits)
    return RT(v.contiguous(), a.bits)


def slice_axis(a: RT, axis: int, start, end, step=None, nb=0) -> RT:
    ax = _ax(a, axis, nb)
    idx = [slice(None)] * a.data.dim()
    idx[ax] = slice(start, end, step)
    return RT(a.data[tuple(idx)].contiguous(), a.bits)


def strided_slice(a: RT, slices, nb=0) -> RT:
    idx = [slice(None)] * nb + list(slices)
    d = a.data
    # torch lacks negative steps: emulate with flip
    for i, s in enumerate(idx):
        if isinstance(s, slice) and s.step is not None and s.step < 0:
            raise NotImplementedError("negative slice steps")
    return RT(d[tuple(idx)].contiguous(), a.bits)


def select_mask(a: RT, axis: int, mask: torch.Tensor, nb=0) -> RT:
    ax = _ax(a, axis, nb)
    keep = torch.nonzero(mask.reshape(-1).to(torch.bool)).reshape(-1).to(a.device)
    return RT(a.data.index_select(ax, keep).contiguous(), a.bits)


def diag(a: RT, nb=0) -> RT:
    d = a.data
    if a.bits == 128:
        return RT(torch.diagonal(d, dim1=nb, dim2=nb + 1).movedim(-1, -2).contiguous(), 128)
    return RT(torch.diagonal(d, dim1=nb, dim2=nb + 1).contiguous(), a.bits)


def broadcast_to(a: RT, shape, nb=0) -> RT:
    shape = tuple(shape)
    lead = len(shape) - (a.ndim - nb)
    if lead > 0:  # numpy rule: missing dims are prepended (after the batch axes)
        a = reshape(a, (1,) * lead + a.shape[nb:], nb)
    return expand(a, a.shape[:nb] + shape).contiguous()


def atleast_2d(a: RT, to_column_vector=False, nb=0) -> RT:
    nd = a.ndim - nb
    if nd >= 2:
        return a
    if nd == 0:
        return reshape(a, (1, 1), nb)
    n = a.shape[nb]
    return reshape(a, (n, 1) if to_column_vector else (1, n), nb)


# ---------------------------------------------------------------------------
# reductions
# ---------------------------------------------------------------------------
def sum(a: RT, axis=None, nb=0) -> RT:  # noqa: A001 - mirrors the Moose op name
    if axis is None:
        # reduce all logical dims
        flat = reshape(a, (a.numel() // max(1, math.prod(a.shape[:nb])),), nb)
        return sum(flat, 0, nb)
    ax = _ax(a, axis, nb)
    if a.bits == 1:
        return RT((a.data.to(torch.int64).sum(dim=ax) & 1).to(torch.uint8), 1)
    if a.bits == 64:
        return RT(a.data.sum(dim=ax), 64)
    shape = a.shape
    outer = math.prod(shape[:ax])
    red = shape[ax]
    inner = math.prod(shape[ax + 1 :])
    out = empty(shape[:ax] + shape[ax + 1 :], 128, a.device)
    ad = a.data.contiguous()
    nat.check(
        nat.lib().mx_sum_axis(
            nat.dev_of(ad), 2, nat.ptr(ad), nat.ptr(out.data), outer, red, inner,
            nat.stream_of(ad),
        ),
        "ring128 sum",
    )
    return out


def add_n(xs: List[RT]) -> RT:
    acc = xs[0]
    for x in xs[1:]:
        acc = acc + x
    return acc


# ---------------------------------------------------------------------------
# GEMM
# ---------------------------------------------------------------------------
def _gemm_call(bits, batch, M, N, K, a0, a1, b0, b1, mode, out, accumulate=0):
    lib = nat.lib()
    limit = (16384 if bits == 64 else 8192) // (2 if mode else 1)
    if out.is_cuda and K > limit:
        # split K so every limb diagonal stays exact in the i32 accumulators
        for k0 in range(0, K, limit):
            k1 = min(K, k0 + limit)
            A0c = _kslice_rows(a0, batch, M, K, k0, k1, bits)
            A1c = _kslice_rows(a1, batch, M, K, k0, k1, bits) if a1 is not None else None
            B0c = _kslice_cols(b0, batch, K, N, k0, k1, bits)
            B1c = _kslice_cols(b1, batch, K, N, k0, k1, bits) if b1 is not None else None
            _gemm_call(bits, batch, M, N, k1 - k0, A0c, A1c, B0c, B1c, mode, out,
                       accumulate if k0 == 0 else 1)
        return
    nat.check(
        lib.mx_gemm(
            nat.dev_of(out), _words(bits), batch, M, N, K, nat.ptr(a0), nat.ptr(a1), nat.ptr(b0),
            nat.ptr(b1), mode, nat.ptr(out), accumulate, nat.stream_of(out),
        ),
        "ring gemm",
    )


def dot_slots(x: RT, c: RT):
    """x[b] . c for every slot b of a device ring tensor x [B, M, K] (or [B, K]) whose slots
    may be any evenly strided views (e.g. the four slots of a share-pair ring buffer) and a
    public operand c [K, N] (or [K]) read by every slot in place -- one launch, no copy of
    c per slot.  None when the layout does not fit (the caller runs R.dot)."""
    d, cd = x.data, c.data
    if (not d.is_cuda or cd.device != d.device or x.bits not in (64, 128)
            or c.bits != x.bits):
        return None
    el = 2 if x.bits == 128 else 1
    xl, cl = tuple(x.shape[1:]), tuple(c.shape)
    if len(xl) == 2 and len(cl) == 2:
        M, K, N, oshape = xl[0], xl[1], cl[1], (xl[0], cl[1])
    elif len(xl) == 2 and len(cl) == 1:
        M, K, N, oshape = xl[0], xl[1], 1, (xl[0],)
    elif len(xl) == 1 and len(cl) == 2:
        M, K, N, oshape = 1, xl[0], cl[1], (cl[1],)
    else:
        return None
    if cl[0] != K or d.stride(0) % el:
        return None
    inner = d[0]
    if not inner.is_contiguous() or not cd.is_contiguous():
        return None
    B = d.shape[0]
    out = empty((B,) + oshape, x.bits, d.device)
    nat.check(nat.lib().mxh_gemm_bs(_words(x.bits), B, M, N, K, nat.ptr(d), d.stride(0) // el,
                                    nat.ptr(cd), 0, nat.ptr(out.data), nat.stream_of(d)),
              "ring gemm (slots)")
    return out


def _kslice_rows(t, batch, M, K, k0, k1, bits):
    v = t.reshape(batch, M, K, -1) if bits == 128 else t.reshape(batch, M, K)
    return v[:, :, k0:k1].contiguous()


def _kslice_cols(t, batch, K, N, k0, k1, bits):
    v = t.reshape(batch, K, N, -1) if bits == 128 else t.reshape(batch, K, N)
    return v[:, k0:k1].contiguous()


def _dot_shapes(xs, ys, nb):
    """Normalise rank-1/2 operands to [batch, M, K] x [batch, K, N]."""
    xl, yl = xs[nb:], ys[nb:]
    bshape = xs[:nb]
    if len(xl) == 1 and len(yl) == 1:
        M, K, N = 1, xl[0], 1
        out = ()
    elif len(xl) == 1:
        M, K, N = 1, xl[0], yl[1]
        out = (N,)
    elif len(yl) == 1:
        M, K, N = xl[0], xl[1], 1
        out = (M,)
    else:
        M, K, N = xl[0], xl[1], yl[1]
        out = (M, N)
    if K != (yl[0]):
        raise ValueError(f"dot shape mismatch {xl} . {yl}")
    return bshape, M, K, N, out


def dot(x: RT, y: RT, nb=0) -> RT:
    """Ring matrix product (np.dot semantics for logical ranks 1/2), batched over nb dims."""
    bits = x.bits
    bshape, M, K, N, oshape = _dot_shapes(x.shape, y.shape, nb)
    batch = math.prod(bshape)
    out = empty(bshape + (M, N), bits, x.device)
    if bits == 1:
        r = (x.data.reshape(batch, M, K).to(torch.int64) @ y.data.reshape(batch, K, N).to(torch.int64)) & 1
        return RT(r.to(torch.uint8).reshape(bshape + oshape), 1)
    a0 = x.data.contiguous()
    b0 = y.data.contiguous()
    _gemm_call(bits, batch, M, N, K, a0, None, b0, None, 0, out.data)
    return reshape(out, oshape, nb) if oshape != (M, N) else out


class PreparedCross:
    """The B' = [y0 + y1; y0] operand of a stacked RSS cross GEMM, limb-split once on the
    device (mx_gemm_prep_b) so that several row blocks of x reuse it (dot_cross_rows).  On
    the host, or when K is too long for one exact chunk, it just keeps y0, y1."""

    def __init__(self, y0: RT, y1: RT):
        self.y0, self.y1, self.bits = y0, y1, y0.bits
        self.batch, self.K, self.N = y0.shape[0], y0.shape[1], y0.shape[2]
        self.lb = None
        if y0.data.is_cuda:
            w = _words(self.bits)
            nbytes = nat.lib().mx_gemm_b_bytes(w, self.batch, self.N, self.K, 1)
            if nbytes > 0:
                d0, d1 = y0.data.contiguous(), y1.data.contiguous()
                self.lb = torch.empty(nbytes, dtype=torch.uint8, device=d0.device)
                nat.check(nat.lib().mx_gemm_prep_b(
                    w, self.batch, self.K, self.N, nat.ptr(d0), nat.ptr(d1), 1,
                    nat.ptr(self.lb), nat.stream_of(d0)), "gemm_prep_b")


def dot_cross_rows(x0: RT, x1: RT, r0: int, r1: int, pb: PreparedCross) -> RT:
    """Rows [r0, r1) of the stacked cross GEMM x0.(y0+y1) + x1.y0 for x* [batch, M, K]
    (no copy of the row block on the device)."""
    if pb.lb is None:
        rows = lambda t: RT(t.data[:, r0:r1], t.bits)  # noqa: E731
        return dot_cross(rows(x0), rows(x1), pb.y0, pb.y1, nb=1)
    batch, M, K = x0.shape
    d0, d1 = x0.data, x1.data
    if not (d0.is_contiguous() and d1.is_contiguous()):
        d0, d1 = d0.contiguous(), d1.contiguous()
    el = 2 if pb.bits == 128 else 1  # int64 words per element
    out = empty((batch, r1 - r0, pb.N), pb.bits, d0.device)
    off = r0 * K * el * 8
    nat.check(nat.lib().mx_gemm_with_b(
        _words(pb.bits), batch, r1 - r0, pb.N, K, ctypes.c_void_p(d0.data_ptr() + off),
        ctypes.c_void_p(d1.data_ptr() + off), M * K, 1,
        nat.ptr(pb.lb), nat.ptr(out.data), 0, nat.stream_of(d0)), "gemm_with_b")
    return out


def dot_cross_pair(x0: RT, y0: RT, y1: RT, roll: int, pb: PreparedCross = None, r0=0,
                   r1=None):
    """dot_cross(x0, x1, y0, y1) for a stacked RSS pair whose second share is the first
    rolled over the flattened batch (x1[b] = x0[(b + roll) % batch]): the CRT GEMM prepares
    each share's residues once and reads them for both K halves.  Rows [r0, r1) of x0 only
    when given.  None when the device path does not apply (the caller runs dot_cross)."""
    d0 = x0.data
    if not d0.is_cuda or len(x0.shape) != 3:
        return None
    if not d0.is_contiguous():
        d0 = d0.contiguous()
    batch, M, K = x0.shape
    r1 = M if r1 is None else r1
    bits = x0.bits
    el = 2 if bits == 128 else 1
    if pb is not None:
        if pb.lb is None:
            return None
        N, lb, b0, b1 = pb.N, nat.ptr(pb.lb), None, None
    else:
        # [batch, K, N] right operands only (a stacked secret vector [batch, K] takes the
        # generic dot_cross path, which handles rank-1 operands)
        if (len(y0.shape) != 3 or tuple(y1.shape) != tuple(y0.shape)
                or y0.shape[0] != batch or y0.shape[1] != K):
            return None
        N = y0.shape[2]
        b0, b1 = y0.data.contiguous(), y1.data.contiguous()
        lb = None
    out = empty((batch, r1 - r0, N), bits, d0.device)
    rc = nat.lib().mx_gemm_roll(
        _words(bits), batch, r1 - r0, N, K, ctypes.c_void_p(d0.data_ptr() + r0 * K * el * 8),
        M * K, roll, None if b0 is None else nat.ptr(b0), None if b1 is None else nat.ptr(b1),
        lb, nat.ptr(out.data), 0, nat.stream_of(d0))
    if rc == -7:
        return None
    nat.check(rc, "gemm_roll")
    return out


def _asym_operands(x0: RT, x1: RT, y0: RT, y1: RT):
    """Stacks (A0, A1, B0, B1) whose mode-1 cross GEMM A0.(B0 + B1) + A1.B0 is the
    asymmetric z_p of dot_cross_asym, per party p with (a, b, c, d) = (x0, x1, y0, y1)[p]:
    (a + b, 0, c, d), (b, a, d, c), (a, b, c, d - c)."""
    def at(t, p):
        return RT(t.data[p], t.bits)

    a, b, c, d = ([at(t, p) for p in range(3)] for t in (x0, x1, y0, y1))
    zero = zeros(tuple(x0.shape[1:]), x0.bits, x0.device)
    stk = lambda ts: RT(torch.stack([t.data for t in ts]), x0.bits)  # noqa: E731
    A0 = stk([binary("add", a[0], b[0]), b[1], a[2]])
    A1 = stk([zero, a[1], b[2]])
    B0 = stk([c[0], d[1], c[2]])
    B1 = stk([d[0], c[1], binary("sub", d[2], c[2])])
    return A0, A1, B0, B1


def dot_cross_asym(x0: RT, x1: RT, y0: RT, y1: RT, rolled: bool = False) -> RT:
    """The three parties' local products of a replicated matrix product, in the asymmetric
    form (x0/x1: [3, M, K] first/second share stacks, y0/y1: [3, K, N]).  With party p
    holding (a, b) = (x_p, x_{p+1}), (c, d) = (y_p, y_{p+1}):

        z_0 = (a + b)(c + d),   z_1 = b (c + d) + a d,   z_2 = a d + b c.

    Every x_i y_j appears exactly once over the three parties, so sum_p z_p = x.y as in the
    symmetric form z_p = a (c + d) + b c (Araki et al.; the reference's
    replicated/arith.rs:436-492), and each z_p is a function of party p's own shares only.
    Party 0's product is one K-long GEMM instead of two: five K-long GEMMs per product
    instead of six.  The zero share added before the reshare masks z_p exactly as before.
    On the device the five run as one CRT GEMM launch (mx_gemm_asym; ``rolled``: x1/y1 are
    x0/y0 rolled by one party, so x_2's residues are shared by parties 1 and 2); elsewhere
    the same z_p by the generic cross GEMM of rearranged operands (_asym_operands)."""
    bits = x0.bits
    M, K = x0.shape[1], x0.shape[2]
    N = y0.shape[2]
    d = x0.data
    if d.is_cuda and bits in (64, 128) and x0.shape[0] == 3 and y0.shape[0] == 3:
        ts = [t.data if t is not None else None for t in (x0, x1, y0, y1)]
        if rolled:
            ts[1] = ts[3] = None
        if all(t is None or t.is_contiguous() for t in ts):
            out = empty((3, M, N), bits, d.device)
            rc = nat.lib().mx_gemm_asym(
                _words(bits), M, N, K, nat.ptr(ts[0]), None if ts[1] is None else nat.ptr(ts[1]),
                nat.ptr(ts[2]), None if ts[3] is None else nat.ptr(ts[3]), 1 if rolled else 0,
                nat.ptr(out.data), nat.stream_of(d))
            if rc != -7:
                nat.check(rc, "gemm_asym")
                return out
    if x1 is None or y1 is None:
        x1 = RT(torch.roll(x0.data, -1, dims=0), bits)
        y1 = RT(torch.roll(y0.data, -1, dims=0), bits)
    A0, A1, B0, B1 = _asym_operands(x0, x1, y0, y1)
    return dot_cross(A0, A1, B0, B1, nb=1)


def _party_batch_strides(t: RT):
    """(party stride, batch stride) in ring elements of a [P, B, *inner] device tensor whose
    inner dims are contiguous (e.g. an expanded, stride-0 stack of one operand); None if
    the layout is anything else."""
    d = t.data
    el = 2 if t.bits == 128 else 1
    if d.dim() < 3:
        return None
    expect = 1
    for size, st in zip(reversed(d.shape[2:]), reversed(d.stride()[2:])):
        if size != 1 and st != expect:
            return None
        expect *= size
    if d.stride(0) % el or d.stride(1) % el:
        return None
    return d.stride(0) // el, d.stride(1) // el


def _dot_cross_strided(x0, x1, y0, y1, out, M, K, N):
    """Per-party strided GEMMs for [3, B, M, K] x [3, B, K, N] operands that are views
    (no copy of an expanded stack).  False when the layout does not allow it."""
    bits = x0.bits
    limit = (16384 if bits == 64 else 8192) // 2
    if not out.data.is_cuda or K > limit:
        return False
    st = [_party_batch_strides(t) for t in (x0, x1, y0, y1)]
    if any(s is None for s in st) or st[0][1] != st[1][1] or st[2][1] != st[3][1]:
        return False
    eb = 16 if bits == 128 else 8
    B = out.shape[1]
    lib = nat.lib()
    for p in range(out.shape[0]):
        def at(t, s):
            return ctypes.c_void_p(t.data.data_ptr() + p * s[0] * eb)
        optr = ctypes.c_void_p(out.data.data_ptr() + p * B * M * N * eb)
        nat.check(lib.mx_gemm_strided(_words(bits), B, M, N, K, at(x0, st[0]), at(x1, st[1]),
                                      st[0][1], at(y0, st[2]), at(y1, st[3]), st[2][1], 1, optr,
                                      0, nat.stream_of(out.data)), "gemm_strided")
    return True


def dot_cross(x0: RT, x1: RT, y0: RT, y1: RT, nb=0) -> RT:
    """RSS cross terms of a matrix product: x0.(y0+y1) + x1.y0 in one K-doubled GEMM."""
    bits = x0.bits
    bshape, M, K, N, oshape = _dot_shapes(x0.shape, y0.shape, nb)
    batch = math.prod(bshape)
    out = empty(bshape + (M, N), bits, x0.device)
    if (nb == 2 and oshape == (M, N) and not all(
            t.data.is_contiguous() for t in (x0, x1, y0, y1))
            and _dot_cross_strided(x0, x1, y0, y1, out, M, K, N)):
        return out
    _gemm_call(
        bits, batch, M, N, K, x0.data.contiguous(), x1.data.contiguous(), y0.data.contiguous(),
        y1.data.contiguous(), 1, out.data,
    )
    return reshape(out, oshape, nb) if oshape != (M, N) else out


# ---------------------------------------------------------------------------
# randomness (AES-128-CTR)
# ---------------------------------------------------------------------------
def prf_expand(keys: Sequence[bytes], nonce: int, shape, bits, device) -> RT:
    """out[p] = PRF(keys[p], nonce) of the given logical shape; stacked over keys."""
    shape = tuple(shape)
    n = math.prod(shape)
    out = empty((len(keys),) + shape, bits, device)
    kb = nat.key_buffer(keys)
    if len(keys) > 4:
        raise ValueError("at most 4 keys per call")
    nat.check(
        nat.lib().mx_prf_expand(
            nat.dev_of(out.data), _words(bits), nat.ptr(out.data), n, len(keys), kb,
            nonce & MASK64, nat.stream_of(out.data),
        ),
        "prf_expand",
    )
    return out


def bit_planes(a: RT, start: int, count: int, nb=0) -> RT:
    """Bits start..start+count-1 of ``a`` as a bit tensor with a new logical leading axis
    (after ``nb`` batch axes): out[.., j, ..] = bit start+j.  One kernel."""
    shp = a.shape
    outer = math.prod(shp[:nb])
    inner = math.prod(shp[nb:])
    out = torch.empty(tuple(shp[:nb]) + (count,) + tuple(shp[nb:]), dtype=torch.uint8,
                      device=a.device)
    ad = a.data.contiguous()
    nat.check(nat.lib().mx_bit_planes(nat.dev_of(ad), _words(a.bits), nat.ptr(ad), nat.ptr(out),
                                      outer, inner, start, count, nat.stream_of(ad)),
              "bit_planes")
    return RT(out, 1)


_WEIGHTS = {}


_CONSTS = {}


def const_ints(values, bits, device) -> RT:
    """A public constant vector of python ints on ``device``, made once per (values, bits,
    device) and shared -- callers never write into it (no upload per evaluation; not
    cached while a hipGraph is being captured: it would live in the graph's pool)."""
    key = (tuple(int(v) for v in values), bits, str(device))
    hit = _CONSTS.get(key)
    if hit is not None:
        return hit
    t = from_ints(np.array(list(key[0]), dtype=object), bits, device)
    if torch.device(device).type == "cpu" or not torch.cuda.is_current_stream_capturing():
        _cache_put(_CONSTS, key, t, 4096)
        if _CONSTS.get(key) is t:  # only what the cache keeps (it is bounded)
            _const_key[id(t)] = key
    return t


_const_key = {}  # id of a cached constant -> its _CONSTS key (constants are never freed)


_LEADING = {}


def mul_leading(a: RT, c: RT, nb: int) -> RT:
    """a[.., i, ..] * c[i] along the first non-batch axis of ``a``: the public vector
    broadcast to a's shape is made once per (constant, shape) when ``c`` is a shared
    constant (const_ints), so an evaluation runs one multiply kernel and no copy."""
    k = len(a.shape) - nb - 1
    cb = reshape(c, (c.shape[0],) + (1,) * k)
    shared = c.data.is_cuda and _CONSTS.get(_const_key.get(id(c))) is c
    if not shared:
        return binary("mul", a, cb)
    key = (id(c), tuple(a.shape))
    full = _LEADING.get(key)
    if full is None:
        full = RT(expand(cb, tuple(a.shape)).data.contiguous(), a.bits)
        if not torch.cuda.is_current_stream_capturing():
            _cache_put(_LEADING, key, full, 1024)
    return binary("mul", a, full)


def mul_leading_add2(a0: RT, a1: RT, c: RT, cadd: RT, add0: bool, add1: bool):
    """One party's two share components scaled by the public vector ``c`` along the leading
    axis (mul_leading, nb = 1) plus the public scalar ``cadd`` on the components flagged
    ``add0`` / ``add1`` (add_public on this party's copies of x_0), one launch
    (mx_mul_add2).  None when the operands do not fit (then the caller runs the steps)."""
    if not (a0.bits in (64, 128) and a1.bits == a0.bits and a1.shape == a0.shape
            and isinstance(cadd, RT) and cadd.bits == a0.bits and cadd.numel() == 1
            and c.bits == a0.bits and len(a0.shape) >= 1 and c.numel() == a0.shape[0]):
        return None
    k = len(a0.shape) - 1
    # the broadcast is cached only for a shared constant (its id stays its own)
    shared = _CONSTS.get(_const_key.get(id(c))) is c
    key = (id(c), tuple(a0.shape), "pair")
    full = _LEADING.get(key) if shared else None
    if full is None:
        full = RT(expand(reshape(c, (c.shape[0],) + (1,) * k), tuple(a0.shape)).data
                  .contiguous(), a0.bits)
        if shared and not (a0.data.is_cuda and torch.cuda.is_current_stream_capturing()):
            _cache_put(_LEADING, key, full, 1024)
    d0, d1 = a0.data.contiguous(), a1.data.contiguous()
    cd = cadd.data.contiguous()
    if cd.device != d0.device:
        cd = cd.to(d0.device)
    o0, o1 = empty2(a0.shape, a0.bits, a0.device)
    nat.check(nat.lib().mx_mul_add2(
        nat.dev_of(d0), _words(a0.bits), nat.ptr(d0), nat.ptr(d1), nat.ptr(full.data),
        nat.ptr(cd), int(bool(add0)), int(bool(add1)), nat.ptr(o0.data), nat.ptr(o1.data),
        a0.numel(), nat.stream_of(d0)), "mul_add2")
    return o0, o1


def mul_leading_add(a: RT, c: RT, nb: int, cadd: RT, rows) -> RT:
    """mul_leading(a, c, nb) plus the public scalar ``cadd`` on batch rows ``rows`` (two of
    a's leading axis) in one launch (k_mul_rows_add); None when mul_leading would not use a
    cached broadcast (then the caller runs the two steps)."""
    if not (a.data.is_cuda and a.bits in (64, 128) and nb == 1 and isinstance(cadd, RT)
            and cadd.bits == a.bits and cadd.numel() == 1):
        return None
    if not (c.data.is_cuda and _CONSTS.get(_const_key.get(id(c))) is c):
        return None
    k = len(a.shape) - nb - 1
    cb = reshape(c, (c.shape[0],) + (1,) * k)
    key = (id(c), tuple(a.shape))
    full = _LEADING.get(key)
    if full is None:
        full = RT(expand(cb, tuple(a.shape)).data.contiguous(), a.bits)
        if not torch.cuda.is_current_stream_capturing():
            _cache_put(_LEADING, key, full, 1024)
    ad = a.data.contiguous()
    cd = cadd.data.contiguous()
    if cd.device != ad.device:
        cd = cd.to(ad.device)
    out = empty(a.shape, a.bits, a.device)
    n = a.numel()
    nat.check(nat.lib().mxh_mul_rows_add(_words(a.bits), nat.ptr(ad), nat.ptr(full.data),
                                         nat.ptr(out.data), n, n // a.shape[0], nat.ptr(cd),
                                         int(rows[0]), int(rows[1]), nat.stream_of(ad)),
              "mul_rows_add")
    return out


def weighted_sum(a: RT, weights, nb=0) -> RT:
    """sum_j weights[j] * a[.., j, ..] over the leading logical axis (public integer
    weights, e.g. bit composition).  One kernel."""
    bits = a.bits
    key = (tuple(int(w) for w in weights), bits, str(a.device))
    w = _WEIGHTS.get(key)
    if w is None:
        w = from_ints(np.array([int(v) for v in weights], dtype=object), bits, a.device)
        if a.device.type == "cpu" or not torch.cuda.is_current_stream_capturing():
            _cache_put(_WEIGHTS, key, w, 4096)
    shp = a.shape
    k = shp[nb]
    outer = math.prod(shp[:nb])
    inner = math.prod(shp[nb + 1:])
    out = empty(tuple(shp[:nb]) + tuple(shp[nb + 1:]), bits, a.device)
    ad = a.data.contiguous()
    nat.check(nat.lib().mx_weighted_sum(nat.dev_of(ad), _words(bits), nat.ptr(ad),
                                        nat.ptr(w.data), nat.ptr(out.data), outer, k, inner,
                                        nat.stream_of(ad)), "weighted_sum")
    return out


def prf_expand_k(slot_ptr: int, nkeys: int, nonce: int, shape, bits, device) -> RT:
    """``prf_expand`` with the keys read from ``nkeys`` consecutive key slots."""
    shape = tuple(shape)
    n = math.prod(shape)
    out = empty((nkeys,) + shape, bits, device)
    nat.check(
        nat.lib().mx_prf_expand_k(
            nat.dev_of(out.data), _words(bits), nat.ptr(out.data), n, nkeys,
            ctypes.c_void_p(slot_ptr), nonce & MASK64, nat.stream_of(out.data),
        ),
        "prf_expand_k",
    )
    return out


def prg_bytes(key: bytes, nonce: int, nbytes: int, device="cpu", ctr0=0) -> torch.Tensor:
    out = torch.empty(nbytes, dtype=torch.uint8, device=device)
    kb = nat.key_buffer([key])
    nat.check(
        nat.lib().mx_prg(nat.dev_of(out), kb, nonce & MASK64, ctr0, nat.ptr(out), nbytes,
                         nat.stream_of(out)),
        "prg",
    )
    return out


def aes_encrypt(key: bytes, block: bytes) -> bytes:
    import ctypes

    kb = nat.key_buffer([key])
    inp = ctypes.create_string_buffer(bytes(block), 16)
    out = ctypes.create_string_buffer(16)
    nat.check(nat.lib().mx_aes_encrypt_blocks(kb, inp, out, 1), "aes")
    return out.raw


def _party_view(t: RT):
    """(party stride, period) in elements of a stacked [3, *inner] operand: element e of
    party p lives at p * ps + e % per.  Covers contiguous data, slices along the first inner
    axis and one row broadcast over it (stride 0); None for anything else."""
    d = t.data
    shape, strides = list(d.shape), list(d.stride())
    if t.bits == 128:
        if shape[-1] != 2 or strides[-1] != 1 or any(st % 2 for st in strides[:-1]):
            return None
        shape, strides = shape[:-1], [st // 2 for st in strides[:-1]]
    inner, ist = shape[1:], strides[1:]

    def dense(sh, st):
        expect = 1
        for size, stride in zip(reversed(sh), reversed(st)):
            if size != 1 and stride != expect:
                return False
            expect *= size
        return True

    if dense(inner, ist):
        return strides[0], math.prod(inner)
    if inner and ist[0] == 0 and dense(inner[1:], ist[1:]):
        return strides[0], math.prod(inner[1:])
    return None


def rss_mul3_k(kind: str, x0: RT, x1: RT, y0: RT, y1: RT, slot_ptr: int, nonce: int):
    """Stacked 3-party product with the reshare fused in: returns (s0, s1) with
    s0[p] = z_p and s1[p] = z_{p+1} (one kernel, see mx_rss_mul3_k)."""
    bits = x0.bits
    shp = x0.shape
    if y0 is not None and y0.shape != shp:
        x0, y0 = _broadcast(x0, y0)
        shp = x0.shape
    # x1/y0/y1 may be None: y0 None -> out = x0 + zero share (then reshared)
    ops = [None if p is None else (p if p.shape == shp else expand(p, shp)) for p in (x0, x1, y0, y1)]
    n = math.prod(shp) // 3
    out0, out1 = empty2(shp, bits, x0.device)
    if x0.data.is_cuda and any(o is not None and not o.data.is_contiguous() for o in ops):
        views = [(n, n) if o is None else _party_view(o) for o in ops]
        if all(v is not None for v in views):  # slices / row broadcasts read in place
            desc = (ctypes.c_int64 * 8)(*[v[0] for v in views], *[v[1] for v in views])
            nat.check(nat.lib().mx_rss_mul3_kv(
                nat.dev_of(out0.data), 1 if kind == "bool" else 0, _words(bits),
                *[nat.ptr(None if o is None else o.data) for o in ops], nat.ptr(out0.data),
                nat.ptr(out1.data), n, ctypes.c_void_p(slot_ptr), nonce & MASK64, desc,
                nat.stream_of(out0.data)), "rss_mul3_kv")
            return out0, out1
    datas = [None if o is None else o.data.contiguous() for o in ops]
    nat.check(
        nat.lib().mx_rss_mul3_k(
            nat.dev_of(out0.data), 1 if kind == "bool" else 0, _words(bits),
            *[nat.ptr(d) for d in datas], nat.ptr(out0.data), nat.ptr(out1.data), n,
            ctypes.c_void_p(slot_ptr), nonce & MASK64, nat.stream_of(out0.data),
        ),
        "rss_mul3_k",
    )
    return out0, out1


def mul_trunc3_k(x0: RT, x1: RT, y0: RT, y1: RT, slot_ptr: int, nmul: int, m: int, nonces,
                 out=None):
    """Fixed-point product of three stacked parties in one kernel on the device
    (mx_mul_trunc3_kv): ``rss_mul3_k(arith)`` + the stacked TruncPr of its result, bitwise
    the same.  ``out``: optional (s0, s1) views with dense party slots to write into.
    Returns (s0, s1), or None when not applicable (host, large or mixed-shape operands)."""
    bits = x0.bits
    if not x0.data.is_cuda or bits not in (64, 128):
        return None
    shp = x0.shape
    ops = (x0, x1, y0, y1)
    if any(o.shape != shp or o.bits != bits for o in ops):
        return None
    n = math.prod(shp) // 3
    if n == 0:
        return None
    views = None
    if any(not o.data.is_contiguous() for o in ops):
        vs = [_party_view(o) for o in ops]
        if any(v is None for v in vs):
            return None
        views = (ctypes.c_int64 * 8)(*[v[0] for v in vs], *[v[1] for v in vs])
    w = 2 if bits == 128 else 1
    if out is None:
        o0, o1 = ring4(shp, bits, x0.device)
        os_ = n
    else:
        o0, o1 = out
        os_ = o0.data.stride(0) // w
        if not (o0.shape == shp and o1.shape == shp and o1.data.stride(0) == o0.data.stride(0)
                and o0.data[0].is_contiguous() and o1.data[0].is_contiguous()):
            return None
    nn = (ctypes.c_uint64 * 6)(*[v & MASK64 for v in nonces])
    rc = nat.lib().mx_mul_trunc3_kv(
        nat.dev_of(o0.data), _words(bits), *[nat.ptr(o.data) for o in ops], nat.ptr(o0.data),
        nat.ptr(o1.data), n, os_, ctypes.c_void_p(slot_ptr), nmul & MASK64, int(m), nn, views,
        nat.stream_of(o0.data))
    if rc == 1:
        return None
    nat.check(rc, "mul_trunc3")
    return o0, o1


def _mt3_args(x0: RT, x1: RT, y0: RT, y1: RT, out=None):
    """mul_trunc3_k's argument checks and layout: (ops, (o0, o1), n, out stride, views) or
    None when the device kernel does not apply."""
    bits = x0.bits
    if not x0.data.is_cuda or bits not in (64, 128):
        return None
    shp = x0.shape
    ops = (x0, x1, y0, y1)
    if any(o.shape != shp or o.bits != bits for o in ops):
        return None
    n = math.prod(shp) // 3
    if n == 0:
        return None
    views = None
    if any(not o.data.is_contiguous() for o in ops):
        vs = [_party_view(o) for o in ops]
        if any(v is None for v in vs):
            return None
        views = [v[0] for v in vs] + [v[1] for v in vs]
    w = 2 if bits == 128 else 1
    if out is None:
        o0, o1 = ring4(shp, bits, x0.device)
        os_ = n
    else:
        o0, o1 = out
        os_ = o0.data.stride(0) // w
        if not (o0.shape == shp and o1.shape == shp and o1.data.stride(0) == o0.data.stride(0)
                and o0.data[0].is_contiguous() and o1.data[0].is_contiguous()):
            return None
    return ops, (o0, o1), n, os_, views


def mul_trunc3_k2(jobs, slot_ptr: int):
    """Two independent fixed-point products of one placement in ONE launch
    (mx_mul_trunc3_kv2): ``jobs`` = [(x0, x1, y0, y1, nmul, m, nonces, out), ...] (two),
    each exactly mul_trunc3_k's.  Returns [(s0, s1), (s0, s1)], or None when the batched
    kernel does not apply (the caller runs them one by one)."""
    if len(jobs) != 2:
        return None
    prep = [_mt3_args(*j[:4], out=j[7]) for j in jobs]
    if any(p is None for p in prep) or jobs[0][0].bits != jobs[1][0].bits:
        return None
    bits = jobs[0][0].bits
    if any(p[2] > 8192 * (16 // (16 if bits == 128 else 8)) for p in prep):
        return None  # throughput sizes: one by one
    P2 = ctypes.c_void_p * 2
    ptr = lambda t: t.data.data_ptr()  # noqa: E731
    vws = [None if p[4] is None else (ctypes.c_int64 * 8)(*p[4]) for p in prep]
    views = (ctypes.c_void_p * 2)(*[None if v is None else ctypes.addressof(v) for v in vws])
    nn = (ctypes.c_uint64 * 12)(*[v & MASK64 for j in jobs for v in j[6]])
    rc = nat.lib().mxh_mul_trunc3_kv2(
        _words(bits), P2(*[ptr(p[0][0]) for p in prep]), P2(*[ptr(p[0][1]) for p in prep]),
        P2(*[ptr(p[0][2]) for p in prep]), P2(*[ptr(p[0][3]) for p in prep]),
        P2(*[ptr(p[1][0]) for p in prep]), P2(*[ptr(p[1][1]) for p in prep]),
        (ctypes.c_int64 * 2)(*[p[2] for p in prep]), (ctypes.c_int64 * 2)(*[p[3] for p in prep]),
        ctypes.c_void_p(slot_ptr), (ctypes.c_uint64 * 2)(*[j[4] & MASK64 for j in jobs]),
        (ctypes.c_int * 2)(*[int(j[5]) for j in jobs]), nn, views,
        nat.stream_of(jobs[0][0].data))
    if rc == -1:
        return None
    nat.check(rc, "mul_trunc3 x2")
    return [p[1] for p in prep]


def zs_trunc3_k(z: RT, slot_ptr: int, nmul: int, m: int, nonces):
    """Zero share + reshare + TruncPr of three stacked parties' local products ``z``
    ([3, ...], e.g. a dot's GEMM output) in one kernel (mx_mul_trunc3_kv with the product
    given): bitwise ``trunc_pr3(rss_mul3_k(arith, z))`` -- the reshared product is never
    written.  Returns (s0, s1), or None on the host."""
    bits = z.bits
    if not z.data.is_cuda or bits not in (64, 128):
        return None
    d = z.data.contiguous()
    shp = z.shape
    n = math.prod(shp) // 3
    if n == 0:
        return None
    o0, o1 = ring4(shp, bits, d.device)
    nn = (ctypes.c_uint64 * 6)(*[v & MASK64 for v in nonces])
    rc = nat.lib().mx_mul_trunc3_kv(
        nat.dev_of(d), _words(bits), nat.ptr(d), None, None, None, nat.ptr(o0.data),
        nat.ptr(o1.data), n, n, ctypes.c_void_p(slot_ptr), nmul & MASK64, int(m), nn, None,
        nat.stream_of(d))
    if rc == 1:
        return None
    nat.check(rc, "zs_trunc3")
    return o0, o1


def zs_trunc3_rows(z: RT, slot_ptr: int, nmul: int, m: int, nonces, buf4, r0: int):
    """zs_trunc3_k for the row block [r0, r0 + rows) of a pipelined product: ``z`` =
    [3, rows, N] local products, the shares written straight into rows of ``buf4`` (the
    result's [4, M, N] share-pair ring buffer, slots x0, x1, x2, x0)."""
    bits = z.bits
    d = z.data.contiguous()
    n = math.prod(z.shape) // 3  # ring elements per party in the block
    el = 2 if bits == 128 else 1
    os_ = math.prod(buf4.shape[1:]) // el  # party stride of the result (elements)
    o0 = buf4.data_ptr() + r0 * math.prod(buf4.shape[2:]) * 8
    nn = (ctypes.c_uint64 * 6)(*[v & MASK64 for v in nonces])
    rc = nat.lib().mx_mul_trunc3_kv(
        nat.dev_of(d), _words(bits), nat.ptr(d), None, None, None, ctypes.c_void_p(o0),
        ctypes.c_void_p(o0 + os_ * el * 8), n, os_, ctypes.c_void_p(slot_ptr), nmul & MASK64,
        int(m), nn, None, nat.stream_of(d))
    nat.check(rc, "zs_trunc3_rows")


def add_zs3(v: RT, r: RT):
    """Stacked arith zero share from precomputed keystreams ``r`` (= PRF(k_p) per party)
    plus the reshare: returns (s0, s1) exactly like ``rss_mul3_k(arith, v)``."""
    vd, rd = v.data.contiguous(), r.data.contiguous()
    n = math.prod(v.shape) // 3
    o0, o1 = empty(v.shape, v.bits, v.device), empty(v.shape, v.bits, v.device)
    nat.check(nat.lib().mx_add_zs3(nat.dev_of(vd), _words(v.bits), nat.ptr(vd), nat.ptr(rd),
                                   nat.ptr(o0.data), nat.ptr(o1.data), n, nat.stream_of(vd)),
              "add_zs3")
    return o0, o1


def _slot_operand_ok(a: RT, b: RT) -> bool:
    """b broadcasts over one slot of stacked a as a period: a scalar, or b's shape (leading
    1s dropped) is a suffix of the slot's shape."""
    if b.numel() == 1:
        return True
    bs = list(b.shape)
    while bs and bs[0] == 1:
        bs.pop(0)
    ss = list(a.shape[1:])
    return len(bs) <= len(ss) and ss[len(ss) - len(bs):] == bs


def binary_slot(op: str, a: RT, b: RT, which: int):
    """Stacked [nparties, *shape] ``a``: ``op`` with public ``b`` (same shape as one slot,
    or a scalar) applied to slot ``which`` only, one kernel (mx_ew_binary_slot)."""
    np_, m = a.shape[0], math.prod(a.shape[1:])
    nb = b.numel()
    if not _slot_operand_ok(a, b):
        raise ValueError("binary_slot: operand must be a scalar, one slot's shape or a "
                         "trailing-axes suffix of it")
    ad = a.data.contiguous()
    bd = b.data.contiguous()
    if bd.device != ad.device:
        bd = bd.to(ad.device)
    out = empty(a.shape, a.bits, a.device)
    nat.check(
        nat.lib().mx_ew_binary_slot(
            nat.dev_of(ad), _BIN[op], _words(a.bits), nat.ptr(ad), nat.ptr(bd), nb,
            nat.ptr(out.data), m, np_, int(which), nat.stream_of(ad),
        ),
        "binary_slot",
    )
    return out


def binary_slot2(op: str, a0: RT, a1: RT, b: RT, which0: int, which1: int):
    """binary_slot on both share vectors (slots which0 / which1) in one launch."""
    if a0.bits == 1 or a1.shape != a0.shape:
        return binary_slot(op, a0, b, which0), binary_slot(op, a1, b, which1)
    np_, m = a0.shape[0], math.prod(a0.shape[1:])
    nb = b.numel()
    if not _slot_operand_ok(a0, b):
        raise ValueError("binary_slot2: operand must be a scalar, one slot's shape or a "
                         "trailing-axes suffix of it")
    d0, d1, bd = a0.data.contiguous(), a1.data.contiguous(), b.data.contiguous()
    if bd.device != d0.device:
        bd = bd.to(d0.device)
    o0, o1 = empty2(a0.shape, a0.bits, a0.device)
    nat.check(nat.lib().mx_ew_binary_slot2(
        nat.dev_of(d0), _BIN[op], _words(a0.bits), nat.ptr(d0), nat.ptr(d1), nat.ptr(bd), nb,
        nat.ptr(o0.data), nat.ptr(o1.data), m, np_, int(which0), int(which1),
        nat.stream_of(d0)), "binary_slot (pair)")
    return o0, o1


_RT_DATA = RT.__dict__["data"]  # the base class's slot descriptor


class Opened(RT):
    """An opened (revealed) value a + b + c [+ d] whose sum is formed on first use of
    ``data``.  A decode of it runs one fused pass (mx_addn_decode) instead of add + decode:
    the ring-valued sum never goes to memory."""

    __slots__ = ("parts", "stream")

    def __init__(self, a: RT, b: RT, c: RT, d: RT = None):
        _RT_DATA.__set__(self, None)
        self.bits = a.bits
        self._shape = a.shape
        self.parts = (a, b, c) if d is None else (a, b, c, d)
        self.stream = _stream_of(a.data)

    def pending(self) -> bool:
        return _RT_DATA.__get__(self) is None

    @property
    def data(self):
        d = _RT_DATA.__get__(self)
        if d is None:
            _join(self.stream)
            s = add3(*self.parts[:3])
            if len(self.parts) == 4:
                s = binary("add", s, self.parts[3])
            d = s.data
            _RT_DATA.__set__(self, d)
            self.parts = None
        return d

    @data.setter
    def data(self, v):
        _RT_DATA.__set__(self, v)

    @property
    def device(self):
        return self.parts[0].device if self.pending() else self.data.device


def opened(a: RT, b: RT, c: RT, d: RT = None) -> RT:
    """a + b + c [+ d] as an :class:`Opened` (lazy) when the fused decode applies.  The
    addends are shares of the value at its own type's scale: a reveal never opens a value
    with more fractional bits than its type (no truncation is ever deferred into a reveal)."""
    parts = (a, b, c) if d is None else (a, b, c, d)
    if a.bits in (64, 128) and all(t.shape == a.shape and t.bits == a.bits for t in parts):
        return Opened(*parts)
    s = add3(a, b, c)
    return s if d is None else binary("add", s, d)


def add3(a: RT, b: RT, c: RT) -> RT:
    """a + b + c of one shape in one pass (mx_ew_add3)."""
    if not (a.shape == b.shape == c.shape and a.bits == b.bits == c.bits) or a.bits == 1:
        return binary("add", binary("add", a, b), c)
    d = [t.data.contiguous() for t in (a, b, c)]
    out = empty(a.shape, a.bits, a.device)
    nat.check(nat.lib().mx_ew_add3(nat.dev_of(d[0]), _words(a.bits), *[nat.ptr(x) for x in d],
                                   nat.ptr(out.data), a.numel(), nat.stream_of(d[0])), "add3")
    return out


def lincomb2(terms, b=None, which0: int = 0, which1: int = 2):
    """Share-wise sum_t coef_t * (s0_t, s1_t) of stacked [nparties, ...] share vectors (+ the
    public ``b`` at slots which0 / which1) in one launch (mx_lincomb2).  ``terms``: up to 3
    (int coef, RT s0, RT s1) of one shape.  Returns (out0, out1)."""
    c0, a0, _ = terms[0]
    bits, shp = a0.bits, a0.shape
    np_, m = shp[0], math.prod(shp[1:])
    datas = []
    for _, x0, x1 in terms:
        datas += [x0.data.contiguous(), x1.data.contiguous()]
    bd = None
    if b is not None:
        bd = b.data.contiguous()
        if bd.device != a0.device:
            bd = bd.to(a0.device)
    o0, o1 = empty2(shp, bits, a0.device)
    ins = (ctypes.c_void_p * len(datas))(*[d.data_ptr() for d in datas])
    coef = (ctypes.c_int64 * len(terms))(*[int(t[0]) for t in terms])
    nat.check(nat.lib().mx_lincomb2(
        nat.dev_of(o0.data), _words(bits), len(terms), ins, coef, nat.ptr(bd),
        b.numel() if b is not None else 0, nat.ptr(o0.data), nat.ptr(o1.data), m, np_,
        int(which0), int(which1), nat.stream_of(o0.data)), "lincomb2")
    return o0, o1


def _even_views(ts):
    """(base tensor, element step, party stride) when the stacked RTs ``ts`` are views of one
    buffer at a constant step with dense party slots; None otherwise."""
    d0 = ts[0].data
    w = 2 if ts[0].bits == 128 else 1
    if d0.dim() < 1 or not d0[0].is_contiguous() or d0.stride(0) % w:
        return None
    es = d0.element_size() * w
    ptrs = [t.data.data_ptr() for t in ts]
    for t in ts:
        d = t.data
        if (d.shape != d0.shape or d.stride() != d0.stride() or d.dtype != d0.dtype
                or d.device != d0.device or t.bits != ts[0].bits):
            return None
    if len(ts) > 1:
        step = ptrs[1] - ptrs[0]
        if step <= 0 or step % es or any(ptrs[i + 1] - ptrs[i] != step for i in range(len(ts) - 1)):
            return None
        step //= es
    else:
        step = 0
    return d0, step, d0.stride(0) // w


def sum_views2(ts0, ts1):
    """(sum of ts0, sum of ts1) -- k stacked share vectors each -- in one launch when both
    lists are evenly spaced views of one buffer (mx_sum_views2); None otherwise."""
    v0, v1 = _even_views(ts0), _even_views(ts1)
    if v0 is None or v1 is None or ts0[0].shape != ts1[0].shape:
        return None
    bits, shp = ts0[0].bits, ts0[0].shape
    o0, o1 = empty2(shp, bits, ts0[0].device)
    np_, m = shp[0], math.prod(shp[1:])
    nat.check(nat.lib().mx_sum_views2(
        nat.dev_of(o0.data), _words(bits), v0[0].data_ptr(), v1[0].data_ptr(), v0[1], v1[1],
        v0[2], v1[2], len(ts0), nat.ptr(o0.data), nat.ptr(o1.data), m, np_,
        nat.stream_of(o0.data)), "sum_views2")
    return o0, o1


def b2a_prep3(b0: RT, b1: RT, ring_bits: int):
    """rep.b2a's local values for three stacked parties in one launch (k_b2a_prep3): P0's
    a = b_0 ^ b_1 as a ring tensor [...] and the trivial sharing of b_2 (slot 2) as a
    pair of [3, ...] party vectors.  None when not on the device."""
    d0, d1 = b0.data, b1.data
    if not d0.is_cuda or ring_bits not in (64, 128) or d0.dtype != torch.uint8 \
            or d1.dtype != torch.uint8 or d0.shape != d1.shape or d0.shape[0] != 3:
        return None
    d0, d1 = d0.contiguous(), d1.contiguous()
    shp = tuple(d0.shape[1:])
    a = empty(shp, ring_bits, d0.device)
    o0, o1 = empty2((3,) + shp, ring_bits, d0.device)
    nat.check(nat.lib().mxh_b2a_prep3(_words(ring_bits), nat.ptr(d0), nat.ptr(d1),
                                      math.prod(shp), nat.ptr(a.data), nat.ptr(o0.data),
                                      nat.ptr(o1.data), nat.stream_of(d0)), "b2a_prep3")
    return a, o0, o1


def b2a3(b0: RT, b1: RT, ring_bits: int, slot_ptr: int, mir: bool, n1: int, nmul: int):
    """The whole of rep.b2a for three stacked parties in one launch (k_b2a3): P0's sharing
    of a = b_0 ^ b_1 (mask nonce n1, key k_0, or k_1 mirrored), its product with the trivial
    sharing of b_2 (zero-share nonce nmul) and A + B - 2 AB.  Returns the (s0, s1) pair of
    [3, ...] arithmetic share vectors, or None when not on the device."""
    d0, d1 = b0.data, b1.data
    if not d0.is_cuda or ring_bits not in (64, 128) or d0.dtype != torch.uint8 \
            or d1.dtype != torch.uint8 or d0.shape != d1.shape or d0.shape[0] != 3:
        return None
    d0, d1 = d0.contiguous(), d1.contiguous()
    o0, o1 = ring4(tuple(d0.shape), ring_bits, d0.device)
    nat.check(nat.lib().mxh_b2a3(_words(ring_bits), nat.ptr(d0), nat.ptr(d1),
                                 math.prod(d0.shape[1:]), nat.ptr(o0.data), nat.ptr(o1.data),
                                 ctypes.c_void_p(slot_ptr), int(bool(mir)), n1 & MASK64,
                                 nmul & MASK64, nat.stream_of(d0)), "b2a3")
    return o0, o1


def b2a3_planes(w0: RT, w1: RT, start: int, count: int, slot_ptr: int, mir: bool, n1: int,
                nmul: int):
    """b2a3 of BitSplit(start, count) of a packed boolean share pair (w0, w1: [3, ...] ring
    words) in one launch, the planes never materialised: (s0, s1) arithmetic [3, count,
    ...] pairs, or None (host)."""
    d0, d1 = w0.data, w1.data
    bits = w0.bits
    if not d0.is_cuda or bits not in (64, 128) or w1.bits != bits or w0.shape != w1.shape \
            or w0.shape[0] != 3 or start < 0 or count < 1 or start + count > bits:
        return None
    d0, d1 = d0.contiguous(), d1.contiguous()
    rest = tuple(w0.shape[1:])
    o0, o1 = ring4((3, count) + rest, bits, d0.device)
    nat.check(nat.lib().mxh_b2a3_planes(
        _words(bits), nat.ptr(d0), nat.ptr(d1), math.prod(rest), int(start), int(count),
        nat.ptr(o0.data), nat.ptr(o1.data), ctypes.c_void_p(slot_ptr), int(bool(mir)),
        n1 & MASK64, nmul & MASK64, nat.stream_of(d0)), "b2a3_planes")
    return o0, o1


def mux3(s0: RT, s1: RT, x0: RT, x1: RT, y0: RT, y1: RT, slot_ptr: int, nonce: int,
         absv: bool = False):
    """rep.mux(s, x, y) = s * (x - y) + y for arithmetic stacked sharings in one launch
    (k_mux3_lat, zero-share nonce ``nonce``); ``absv``: x - 2 s x instead (y = x, unused).
    Returns (s0, s1), or None (host, shapes)."""
    ts = (s0, s1, x0, x1, y0, y1)
    bits = s0.bits
    if not s0.data.is_cuda or bits not in (64, 128) or any(
            t.bits != bits or t.shape != s0.shape for t in ts) or s0.shape[0] != 3:
        return None
    ds = [t.data.contiguous() for t in ts]
    o0, o1 = ring4(s0.shape, bits, ds[0].device)
    nat.check(nat.lib().mxh_mux3(_words(bits), *[nat.ptr(d) for d in ds], nat.ptr(o0.data),
                                 nat.ptr(o1.data), math.prod(s0.shape[1:]),
                                 ctypes.c_void_p(slot_ptr), nonce & MASK64, int(bool(absv)),
                                 nat.stream_of(ds[0])), "mux3")
    return o0, o1


def bitdec3(x0: RT, x1: RT, slot_ptr: int, mir: bool, n1: int, nmul: int, nonces,
            sign_nonces=None):
    """The whole of rep.bit_decompose for three stacked parties in one launch (k_bitdec3):
    P0's boolean sharing of y = x_0 + x_1 (mask nonce n1, key k_0 or mirrored k_1), the
    trivial sharing of x_2, the adder's xor and AND (zero-share nonce nmul) and its
    Kogge-Stone chain (``nonces``, one per level) with the sum.  Returns the (s0, s1) pair of
    packed boolean share vectors [3, ...], or None (host, or above the latency sizes).
    ``sign_nonces`` = (n1', nmul'): instead, the b2a of the sum's top bit (rep.b2a of
    rep.msb: its sharing and product nonces) as an arithmetic share pair."""
    d0, d1 = x0.data, x1.data
    bits = x0.bits
    if not d0.is_cuda or bits not in (64, 128) or x1.bits != bits or x0.shape != x1.shape \
            or x0.shape[0] != 3:
        return None
    n = math.prod(x0.shape[1:])
    if n > 65536 or len(nonces) != bits.bit_length() - 1:
        return None
    d0, d1 = d0.contiguous(), d1.contiguous()
    sign = sign_nonces is not None
    o0, o1 = (ring4 if sign else empty2)(x0.shape, bits, d0.device)
    arr = (ctypes.c_uint64 * len(nonces))(*[int(v) & MASK64 for v in nonces])
    sb = sign_nonces or (0, 0)
    rc = nat.lib().mxh_bitdec3(_words(bits), nat.ptr(d0), nat.ptr(d1), nat.ptr(o0.data),
                               nat.ptr(o1.data), n, len(nonces), ctypes.c_void_p(slot_ptr),
                               int(bool(mir)), n1 & MASK64, nmul & MASK64, arr, int(sign),
                               sb[0] & MASK64, sb[1] & MASK64, nat.stream_of(d0))
    nat.check(rc, "bitdec3")
    return o0, o1


def slot_place2(x0: RT, x1: RT, which0: int, which1: int, nparties: int = 3):
    """Two trivial stacked sharings [nparties, *x.shape] in one launch: slot which0 of the
    first = x0, slot which1 of the second = x1, zeros elsewhere (mx_slot_place2)."""
    bits = x0.bits
    shp = (nparties,) + tuple(x0.shape)
    o0, o1 = empty2(shp, bits, x0.device)
    d0, d1 = x0.data.contiguous(), x1.data.contiguous()
    nat.check(nat.lib().mx_slot_place2(
        nat.dev_of(d0), _words(bits), nat.ptr(d0), nat.ptr(d1), nat.ptr(o0.data),
        nat.ptr(o1.data), x0.numel(), nparties, int(which0), int(which1), nat.stream_of(d0)),
        "slot_place2")
    return o0, o1


def ks_cross1(g0: RT, g1: RT, p0: RT, p1: RT, d: int, both: bool, keys, nonce: int) -> RT:
    """One party's masked cross terms of a Kogge-Stone level (mx_ks_cross1): shape
    ``[2, *shape]`` (t, pk') if ``both`` else ``shape``; ``keys`` = (k_p, k_{p+1})."""
    bits = g0.bits
    shp = g0.shape
    datas = [x.data.contiguous() for x in (g0, g1, p0, p1)]
    n = math.prod(shp)
    z = empty(((2,) + tuple(shp)) if both else tuple(shp), bits, g0.device)
    kbuf = nat.key_buffer(list(keys))
    nat.check(
        nat.lib().mx_ks_cross1(
            nat.dev_of(z.data), _words(bits), *[nat.ptr(x) for x in datas], nat.ptr(z.data),
            n, int(d), 1 if both else 0, kbuf, nonce & MASK64, nat.stream_of(z.data),
        ),
        "ks_cross1",
    )
    return z


def _empty_in(alloc, shape, bits, device) -> RT:
    """``empty``, or from ``alloc(shape, dtype)`` (a session's outbox: a message)."""
    if alloc is None:
        return empty(shape, bits, device)
    shape = tuple(shape)
    if bits == 128:
        return RT(alloc(shape + (2,), torch.int64), 128)
    return RT(alloc(shape, torch.int64 if bits == 64 else torch.uint8), bits)


def ks_cross1_s(g0: RT, g1: RT, p0: RT, p1: RT, d: int, both: bool, slot_ptrs,
                nonce: int, alloc=None) -> RT:
    """ks_cross1 with the keys (k_p, k_{p+1}) read from two device key slots (``alloc``:
    where z, the level's message, goes)."""
    bits = g0.bits
    shp = g0.shape
    datas = [x.data.contiguous() for x in (g0, g1, p0, p1)]
    n = math.prod(shp)
    z = _empty_in(alloc, ((2,) + tuple(shp)) if both else tuple(shp), bits, g0.device)
    nat.check(
        nat.lib().mx_ks_cross1_s(
            nat.dev_of(z.data), _words(bits), *[nat.ptr(x) for x in datas], nat.ptr(z.data),
            n, int(d), 1 if both else 0, _slots_arr(slot_ptrs), nonce & MASK64,
            nat.stream_of(z.data),
        ),
        "ks_cross1_s",
    )
    return z


def ks_cross1x_s(g0: RT, g1: RT, t0, t1, p0: RT, p1: RT, d: int, both: bool, slot_ptrs,
                 nonce: int, alloc=None):
    """ks_cross1_s on g ^ t (the previous level's xor folded into this level's launch;
    t0 = t1 = None: plain ks_cross1_s).  Returns (z, (g0 ^ t0, g1 ^ t1) or None)."""
    if t0 is None:
        return ks_cross1_s(g0, g1, p0, p1, d, both, slot_ptrs, nonce, alloc=alloc), None
    bits = g0.bits
    shp = g0.shape
    datas = [x.data.contiguous() for x in (g0, g1, t0, t1, p0, p1)]
    n = math.prod(shp)
    z = _empty_in(alloc, ((2,) + tuple(shp)) if both else tuple(shp), bits, g0.device)
    go0, go1 = empty2(shp, bits, g0.device)
    nat.check(
        nat.lib().mx_ks_cross1x_s(
            nat.dev_of(z.data), _words(bits), *[nat.ptr(x) for x in datas[:4]],
            nat.ptr(go0.data), nat.ptr(go1.data), nat.ptr(datas[4]), nat.ptr(datas[5]),
            nat.ptr(z.data), n, int(d), 1 if both else 0, _slots_arr(slot_ptrs),
            nonce & MASK64, nat.stream_of(z.data),
        ),
        "ks_cross1x_s",
    )
    return z, (go0, go1)


def ks_sum2(p0: RT, p1: RT, g0: RT, g1: RT, t0: RT, t1: RT):
    """The adder's sum after its last level for both share components, one launch:
    p ^ ((g ^ t) << 1) (mx_ks_sum2)."""
    bits = p0.bits
    datas = [x.data.contiguous() for x in (p0, p1, g0, g1, t0, t1)]
    o0, o1 = empty2(p0.shape, bits, p0.device)
    nat.check(nat.lib().mx_ks_sum2(
        nat.dev_of(o0.data), _words(bits), *[nat.ptr(x) for x in datas], nat.ptr(o0.data),
        nat.ptr(o1.data), math.prod(p0.shape), nat.stream_of(o0.data)), "ks_sum2")
    return o0, o1


def ks_adder3_k(g0: RT, g1: RT, p0: RT, p1: RT, slot_ptr: int, nonces,
                sum_out: bool = False) -> tuple:
    """The whole Kogge-Stone carry chain (len(nonces) levels d = 1, 2, 4, ...) for three
    stacked parties in one launch (mx_ks_adder3_k): bitwise the chain of ks_level3_k calls
    with those nonces; returns the final (g0, g1) -- or, with ``sum_out`` (device only),
    the adder's sum p ^ (g << 1) (p = the initial p0, p1)."""
    bits = g0.bits
    datas = [x.data.contiguous() for x in (g0, g1, p0, p1)]
    n = math.prod(g0.shape) // 3
    o0, o1 = empty2(g0.shape, bits, g0.device)
    arr = (ctypes.c_uint64 * len(nonces))(*[int(v) & MASK64 for v in nonces])
    if sum_out:
        nat.check(nat.lib().mxh_ks_adder3_sum(
            _words(bits), *[nat.ptr(x) for x in datas], nat.ptr(o0.data), nat.ptr(o1.data), n,
            len(nonces), ctypes.c_void_p(slot_ptr), arr, nat.stream_of(o0.data), 1),
            "ks_adder3 (sum)")
        return o0, o1
    nat.check(nat.lib().mx_ks_adder3_k(
        nat.dev_of(o0.data), _words(bits), *[nat.ptr(x) for x in datas], nat.ptr(o0.data),
        nat.ptr(o1.data), n, len(nonces), ctypes.c_void_p(slot_ptr), arr,
        nat.stream_of(o0.data)), "ks_adder3_k")
    return o0, o1


def ks_level3_k(g0: RT, g1: RT, p0: RT, p1: RT, d: int, both: bool, slot_ptr: int,
                nonce: int):
    """One fused Kogge-Stone level for three stacked parties (mx_ks_level3_k): returns
    the reshared (g0', g1', p0', p1') -- p0'/p1' are None unless ``both``."""
    bits = g0.bits
    shp = g0.shape
    datas = [x.data.contiguous() for x in (g0, g1, p0, p1)]
    n = math.prod(shp) // 3
    nout = 4 if both else 2
    blk = empty((nout,) + tuple(shp), bits, g0.device).data
    outs = [RT(blk[i], bits) for i in range(nout)]
    dummy = outs[0].data
    nat.check(
        nat.lib().mx_ks_level3_k(
            nat.dev_of(outs[0].data), _words(bits), *[nat.ptr(x) for x in datas],
            nat.ptr(outs[0].data), nat.ptr(outs[1].data),
            nat.ptr(outs[2].data if both else dummy), nat.ptr(outs[3].data if both else dummy),
            n, int(d), 1 if both else 0, ctypes.c_void_p(slot_ptr), nonce & MASK64,
            nat.stream_of(outs[0].data),
        ),
        "ks_level3_k",
    )
    return (outs[0], outs[1], outs[2], outs[3]) if both else (outs[0], outs[1], None, None)


def rss_cross_k(kind: str, x0: RT, x1, y0, y1, slot_ptr: int, nslots: int, nonce: int,
                nparties: int) -> RT:
    """``rss_cross`` with the zero-share keys read from key slots: party p uses slots
    p % nslots and (p + 1) % nslots."""
    return rss_cross(kind, x0, x1, y0, y1, None, nonce, nparties, _slots=(slot_ptr, nslots))


def rss_cross_kp(kind: str, x0: RT, x1, y0, y1, slot_ptrs, nonce: int) -> RT:
    """``rss_cross`` for stacked parties with independent key PAIRS: party p masks with
    PRF(slot_ptrs[2p]) - PRF(slot_ptrs[2p+1]) (``len(slot_ptrs) == 2 * nparties``).  The
    parties of one stack may then belong to different sessions (mx_rss_cross_kp)."""
    nparties = len(slot_ptrs) // 2
    bits = x0.bits
    shp = x0.shape
    if y0 is not None and y0.shape != shp:
        x0, y0 = _broadcast(x0, y0)
        shp = x0.shape
    datas = [None if p is None else (p if p.shape == shp else expand(p, shp)).data.contiguous()
             for p in (x0, x1, y0, y1)]
    n = math.prod(shp) // nparties
    out = empty(shp, bits, x0.device)
    arr = (ctypes.c_void_p * len(slot_ptrs))(*slot_ptrs)
    nat.check(
        nat.lib().mx_rss_cross_kp(
            nat.dev_of(out.data), 1 if kind == "bool" else 0, _words(bits),
            *[nat.ptr(d) for d in datas], nat.ptr(out.data), n, nparties, arr,
            nonce & MASK64, nat.stream_of(out.data),
        ),
        "rss_cross_kp",
    )
    return out


def rss_cross(kind: str, x0: RT, x1, y0: RT, y1, keys, nonce: int, nparties: int,
              _slots=None) -> RT:
    """Fused RSS local step.  Stacked layout: x* are [nparties, *shape]; party p gets
    x0*y0 + x0*y1 + x1*y0 + PRF(k_p) - PRF(k_{p+1}) (boolean: & / ^).  ``keys`` is a list
    of nparties+1 keys (or None for no zero share)."""
    bits = x0.bits
    shp = x0.shape
    if y0 is not None and y0.shape != shp:
        x0, y0 = _broadcast(x0, y0)
        shp = x0.shape
    parts = [x0, x1, y0, y1]
    datas = []
    for p in parts:
        if p is None:
            datas.append(None)
        else:
            if p.shape != shp:
                p = expand(p, shp)
            datas.append(p.data.contiguous())
    n_total = math.prod(shp)
    n = n_total // nparties
    out = empty(shp, bits, x0.device)
    if _slots is not None:
        nat.check(
            nat.lib().mx_rss_cross_k(
                nat.dev_of(out.data), 1 if kind == "bool" else 0, _words(bits),
                nat.ptr(datas[0]), nat.ptr(datas[1]), nat.ptr(datas[2]), nat.ptr(datas[3]),
                nat.ptr(out.data), n, nparties, ctypes.c_void_p(_slots[0]), _slots[1],
                nonce & MASK64, nat.stream_of(out.data),
            ),
            "rss_cross_k",
        )
        return out
    kbuf = nat.key_buffer(keys) if keys is not None else None
    nat.check(
        nat.lib().mx_rss_cross(
            nat.dev_of(out.data), 1 if kind == "bool" else 0, _words(bits),
            nat.ptr(datas[0]), nat.ptr(datas[1]), nat.ptr(datas[2]), nat.ptr(datas[3]),
            nat.ptr(out.data), n, nparties, kbuf, nonce & MASK64, nat.stream_of(out.data),
        ),
        "rss_cross",
    )
    return out


def zero_share(kind: str, shape, bits, keys, nonce: int, nparties: int, device) -> RT:
    shape = tuple(shape)
    out = empty(shape, bits, device)
    n = math.prod(shape) // nparties
    nat.check(
        nat.lib().mx_zero_share(
            nat.dev_of(out.data), 1 if kind == "bool" else 0, _words(bits), nat.ptr(out.data), n,
            nparties, nat.key_buffer(keys), nonce & MASK64, nat.stream_of(out.data),
        ),
        "zero_share",
    )
    return out


# ---------------------------------------------------------------------------
# per-party protocol rounds (parties of a session on different GPUs)
# ---------------------------------------------------------------------------
def _roles_arr(roles):
    return (ctypes.c_int * len(roles))(*roles)


def _slots_arr(slots):
    return (ctypes.c_void_p * len(slots))(*slots)


def _nonces_arr(nonces):
    return (ctypes.c_uint64 * len(nonces))(*[v & MASK64 for v in nonces])


def trunc_party_r0(s0: RT, s1: RT, m: int, roles, slots, nonces, alloc=None):
    """Round 0 of the per-party TruncPr (mx_trunc_party_r0) on stacked [ncomp, ...] shares.
    Returns (msg, msg_rm, out0, out1): outgoing messages and the (partly filled) new
    shares.  ``alloc``: where the messages go."""
    ncomp = len(roles)
    d0 = s0.data.contiguous()
    d1 = s1.data.contiguous()
    n = math.prod(s0.shape) // ncomp
    msg = _new(alloc, d0.shape, d0.dtype, d0.device)
    out0, out1 = torch.empty_like(d0), torch.empty_like(d0)
    msg_rm = _new(alloc, (ncomp, n), torch.int64, d0.device)
    nat.check(nat.lib().mx_trunc_party_r0(
        nat.dev_of(d0), _words(s0.bits), n, m, ncomp, _roles_arr(roles), nat.ptr(d0),
        nat.ptr(d1), nat.ptr(msg), nat.ptr(msg_rm), nat.ptr(out0), nat.ptr(out1),
        _slots_arr(slots), _nonces_arr(nonces), nat.stream_of(d0)), "trunc_party_r0")
    return msg, msg_rm, out0, out1


def trunc_party_r1(msg, rmk, rrt, rrm, out0, out1, bits, m, roles, slots, nonces,
                   alloc=None):
    """Round 1 (mx_trunc_party_r1): returns w; writes P0's s0 / P1's s1 into out0/out1."""
    ncomp = len(roles)
    n = msg.numel() // ncomp // (2 if bits == 128 else 1)
    w = _new(alloc, msg.shape, msg.dtype, msg.device)
    nat.check(nat.lib().mx_trunc_party_r1(
        nat.dev_of(msg), _words(bits), n, m, ncomp, _roles_arr(roles), nat.ptr(msg),
        nat.ptr(rmk), nat.ptr(rrt), nat.ptr(rrm), nat.ptr(w), nat.ptr(out0), nat.ptr(out1),
        _slots_arr(slots), _nonces_arr(nonces), nat.stream_of(msg)), "trunc_party_r1")
    return w


SHARE_MIRROR = 8  # MX_SHARE_MIRROR (moosex.h): the masked slot goes to P_{j+2}


def share_party(kind: str, x: RT, ncomp: int, rel, slots, n1: int, na: int, mirror=False,
                alloc=None, msg_slot=None):
    """Per-component slots of a sharing by member j (mx_share_party); the owner's out1
    (slot x_{j+1}) is the message to P_{j+1} (whose out0 it becomes).  A pending
    :class:`Encoded` input is encoded inside the kernel.  ``alloc``: two separate buffers
    (a receiver lands its slot whole), slot ``msg_slot`` (the owner's message) from
    ``alloc(shape, dtype)``."""
    code, xd, aux = share_source(x, kind)
    na = na if aux is None else aux
    if alloc is None:
        out0, out1 = empty2((ncomp,) + tuple(x.shape), x.bits, xd.device)
        out0, out1 = out0.data, out1.data
    else:
        out0, out1 = (_empty_in(alloc if s == msg_slot else None, (ncomp,) + tuple(x.shape),
                                x.bits, xd.device).data for s in (0, 1))
    nat.check(nat.lib().mx_share_party(
        nat.dev_of(xd), code | (SHARE_MIRROR if mirror else 0), _words(x.bits), x.numel(), ncomp,
        _roles_arr(rel), nat.ptr(xd), nat.ptr(out0), nat.ptr(out1), _slots_arr(slots),
        n1 & MASK64, na & MASK64, nat.stream_of(xd)), "share_party")
    return out0, out1


# ---------------------------------------------------------------------------
# fixed-point dot tail, per party (csrc/rss_party.hip; moose_amd/parallel/party.py)
# ---------------------------------------------------------------------------
def _vp(ts):
    """Per-component pointer array (None -> null) of dense tensors."""
    for t in ts:
        if t is not None and not t.is_contiguous():
            raise ValueError("per-component buffers must be dense")
    return (ctypes.c_void_p * len(ts))(*[None if t is None else t.data_ptr() for t in ts])


def _dev_stream(ts):
    t = next(t for t in ts if t is not None)
    return nat.dev_of(t), nat.stream_of(t)


def _new(alloc, shape, dtype, device):
    """A message buffer: from ``alloc(shape, dtype)`` (a session's outbox, where the
    receiver reads it in place) or fresh."""
    if alloc is not None:
        return alloc(tuple(shape), dtype)
    return torch.empty(tuple(shape), dtype=dtype, device=device)


def dot_tail_r0(cross, bits, m, roles, slots, nonces, out0, out1, n, dealer=True,
                alloc=None):
    """Round 0 of the per-party dot tail (mx_dot_tail_r0): returns the per-component
    outgoing messages (P0 m0, P1 m1, P2 z2), the dealer's rt1 and rm1 (P2 only); writes
    P2's new shares into out0 / out1.  ``dealer=False``: the dealer's part already ran
    (:func:`dot_tail_dealer`), rt / rm are None.  ``alloc``: where the messages go."""
    msg = [_new(alloc, x.shape, x.dtype, x.device) for x in cross]
    rt = [_new(alloc, x.shape, x.dtype, x.device) if r == 2 and dealer else None
          for x, r in zip(cross, roles)]
    rm = [_new(alloc, (n,), torch.int64, x.device) if r == 2 and dealer else None
          for x, r in zip(cross, roles)]
    dev, st = _dev_stream(cross)
    nat.check(nat.lib().mx_dot_tail_r0(
        dev, _words(bits), n, m, len(roles), _roles_arr(roles), _vp(cross), _vp(msg), _vp(rt),
        _vp(rm), _vp(out0), _vp(out1), _slots_arr(slots), _nonces_arr(nonces), st),
        "dot_tail_r0")
    return msg, rt, rm


def dot_tail_dealer(bits, m, roles, slots, nonces, out0, out1, n, alloc=None):
    """The dealer P2's part of round 0 on its own (mx_dot_tail_r0 without the products):
    it depends on PRF keys and nonces only, so it runs before the product exists and its
    messages rt1 / rm1 travel while the GEMM runs.  Returns (rt, rm) per component (P2's
    components only); writes P2's new shares into out0 / out1."""
    like = [o if r == 2 else None for o, r in zip(out0, roles)]
    rt = [_new(alloc, o.shape, o.dtype, o.device) if o is not None else None for o in like]
    rm = [_new(alloc, (n,), torch.int64, o.device) if o is not None else None for o in like]
    if not any(o is not None for o in like):
        return rt, rm
    only = [r if r == 2 else -1 for r in roles]
    none = [None] * len(roles)
    dev, st = _dev_stream(like)
    nat.check(nat.lib().mx_dot_tail_r0(
        dev, _words(bits), n, m, len(roles), _roles_arr(only), _vp(none), _vp(none), _vp(rt),
        _vp(rm), _vp(out0), _vp(out1), _slots_arr(slots), _nonces_arr(nonces), st),
        "dot_tail_dealer")
    return rt, rm


def dot_tail_r1(msg, rmk, rz, rrt, rrm, bits, m, roles, slots, nonces, out0, out1, n,
                alloc=None):
    """Round 1 (mx_dot_tail_r1): returns w per component (P0, P1); writes P0's s0 and
    P1's s1 into out0 / out1."""
    w = [_new(alloc, x.shape, x.dtype, x.device) if r in (0, 1) else None
         for x, r in zip(msg, roles)]
    dev, st = _dev_stream(msg)
    nat.check(nat.lib().mx_dot_tail_r1(
        dev, _words(bits), n, m, len(roles), _roles_arr(roles), _vp(msg), _vp(rmk), _vp(rz),
        _vp(rrt), _vp(rrm), _vp(w), _vp(out0), _vp(out1), _slots_arr(slots),
        _nonces_arr(nonces), st), "dot_tail_r1")
    return w


def dot_tail_r2(a, b, out, bits, roles, n):
    """out[c] = a[c] + b[c] for the components of P0 and P1 (mx_dot_tail_r2)."""
    if not any(t is not None for t in out):
        return
    dev, st = _dev_stream([t for t in out if t is not None])
    nat.check(nat.lib().mx_dot_tail_r2(dev, _words(bits), n, len(roles), _roles_arr(roles),
                                       _vp(a), _vp(b), _vp(out), st), "dot_tail_r2")


# ---------------------------------------------------------------------------
# the per-party tail over several products at once (csrc/rss_jobs.hip)
# ---------------------------------------------------------------------------
MAX_JOBS = 4


class MulJob:
    """One product of a batched per-party tail: ``rows`` rows of length L (the call's row
    length) with value[r] = cb (x0 y0 + x0 y1 + x1 y0)[r] + ca a[r] + ca2 a2[r], where
    operand rows are read at ``r * stride`` (stride 0: one row broadcast to every row) and
    a / a2 are additive shares (e.g. a party's first share component); the new shares are
    written to the dense rows ``o0`` / ``o1``.  Operands are ring-tensor data (torch)."""

    __slots__ = ("x0", "x1", "y0", "y1", "a", "a2", "o0", "o1", "rows", "sx", "sy", "sa",
                 "sa2", "ca", "ca2", "cb")

    def __init__(self, rows, o0, o1, x=None, y=None, sx=0, sy=0, a=None, sa=0, ca=1, cb=1,
                 a2=None, sa2=0, ca2=1):
        self.rows, self.o0, self.o1 = rows, o0, o1
        self.x0, self.x1 = x if x is not None else (None, None)
        self.y0, self.y1 = y if y is not None else (None, None)
        self.sx, self.sy, self.a, self.sa, self.a2, self.sa2 = sx, sy, a, sa, a2, sa2
        self.ca, self.ca2, self.cb = ca, ca2, (cb if x is not None else 0)


def _jobs_abi(jobs):
    if not 1 <= len(jobs) <= MAX_JOBS:
        raise ValueError(f"1..{MAX_JOBS} jobs per call, got {len(jobs)}")
    ptrs, dims = [], []
    for j in jobs:
        for t in (j.x0, j.x1, j.y0, j.y1, j.a, j.a2, j.o0, j.o1):
            ptrs.append(None if t is None else t.data_ptr())
        for v in (j.rows, j.sx, j.sy, j.sa, j.sa2, j.ca, j.ca2, j.cb):
            v = int(v)
            dims.append(v - (1 << 64) if v >= (1 << 63) else v)
    return (ctypes.c_void_p * len(ptrs))(*ptrs), (ctypes.c_int64 * len(dims))(*dims)


def jobs_r0(jobs, L, bits, m, role, slots, nonces, like, main=True, dealer=True, pend=None,
            alloc=None):
    """Round 0 of the batched per-party tail (mx_jobs_r0): the outgoing message over the
    concatenation of the jobs' rows (P0 m0, P1 m1, P2 z2), the dealer's rt1 / rm1 (P2, when
    ``dealer``), P2's new shares into the jobs' outputs.  ``like``: any tensor of the call's
    device (allocation and stream).  ``pend``: the previous level's round-2 sums still
    pending, [(o, a, b)] with o = a + b elementwise (flat tensors of equal size): operands
    are read through them and they are written too (mx_jobs_r0p)."""
    n = builtins.sum(j.rows for j in jobs) * L
    w = _words(bits)
    shp = (n,) + ((2,) if bits == 128 else ())
    # ``alloc(shape)``: where the outgoing messages go (a session's outbox), else fresh
    new = alloc or (lambda s: torch.empty(s, dtype=torch.int64, device=like.device))
    msg = new(shp) if main else None
    rt = new(shp) if role == 2 and dealer else None
    rm = new((n,)) if role == 2 and dealer else None
    p, d = _jobs_abi(jobs)
    pend = pend or []
    pp = (ctypes.c_void_p * max(1, 3 * len(pend)))(*[t.data_ptr() for r in pend for t in r])
    pl = (ctypes.c_int64 * max(1, len(pend)))(*[r[0].numel() // (2 if bits == 128 else 1)
                                                 for r in pend])
    nat.check(nat.lib().mx_jobs_r0p(
        nat.dev_of(like), w, len(jobs), p, d, L, m, role, int(main), int(dealer),
        None if msg is None else msg.data_ptr(), None if rt is None else rt.data_ptr(),
        None if rm is None else rm.data_ptr(), _slots_arr(slots), _nonces_arr(nonces),
        len(pend), pp, pl, nat.stream_of(like)), "jobs_r0")
    return msg, rt, rm


def jobs_r1(jobs, L, bits, m, role, slots, nonces, msg, rmk, rz, rrt, rrm, alloc=None):
    """Round 1 (mx_jobs_r1): P0 / P1 open c from their message, the other's and z2; returns
    w (P0 w0, P1 w1; None for P2) and writes P0's o0 = z0, P1's o1 = z2.  ``alloc``: where
    w goes (the session's outbox)."""
    if role == 2:
        return None
    w = alloc(tuple(msg.shape)) if alloc is not None else torch.empty_like(msg)
    p, d = _jobs_abi(jobs)
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    nat.check(nat.lib().mx_jobs_r1(
        nat.dev_of(msg), _words(bits), len(jobs), p, d, L, m, role, ptr(msg), ptr(rmk), ptr(rz),
        ptr(rrt), ptr(rrm), w.data_ptr(), _slots_arr(slots), _nonces_arr(nonces),
        nat.stream_of(msg)), "jobs_r1")
    return w


def jobs_r2(jobs, L, bits, role, a, b):
    """Round 2 (mx_jobs_r2): P0's o1 / P1's o0 = w0 + w1."""
    if role == 2:
        return
    p, d = _jobs_abi(jobs)
    nat.check(nat.lib().mx_jobs_r2(nat.dev_of(a), _words(bits), len(jobs), p, d, L, role,
                                   a.data_ptr(), b.data_ptr(), nat.stream_of(a)), "jobs_r2")


# ---------------------------------------------------------------------------
# per-party bit decomposition front and B2A (csrc/rss_bits_party.hip, bits_party.h)
# ---------------------------------------------------------------------------
def _p(t):
    return None if t is None else t.data_ptr()


def bits_front(role, xa, xb, arecv, bits, slots, n1, ng, alloc=None):
    """This party's adder inputs of the bit decomposition of (xa, xb) (its two arithmetic
    components, torch data): (message a1 (P0) or None, z (its zero-shared AND term, the
    reshare message), p0, p1.  ``alloc``: where the messages go)."""
    like = next(t for t in (xa, xb, arecv) if t is not None)
    n = like.numel() // (2 if bits == 128 else 1)
    p0, p1 = torch.empty_like(like), torch.empty_like(like)
    msg = _new(alloc, like.shape, like.dtype, like.device) if role == 0 else None
    z = _new(alloc, like.shape, like.dtype, like.device)
    nat.check(nat.lib().mx_bits_front(
        nat.dev_of(like), _words(bits), role, n, _p(xa), _p(xb), _p(arecv), _p(msg), _p(z),
        _p(p0), _p(p1), _slots_arr(slots), _nonces_arr((n1, ng)), nat.stream_of(like)),
        "bits_front")
    return msg, z, p0, p1


def bits_b2a(phase, role, src, start, count, bits, slots, n1, ng, arecv=None, state=None,
             xbit=-1, blocks=1, alloc=None):
    """B2A of bit planes start.. of a boolean sharing (src = (s0, s1, g0, g1, t0, t1) torch
    data of one party; g = None: s are the sum words), phases 0 / 1 / 2 (bits_party.h).
    ``xbit`` >= 0: rows 0..count-2 are planes start.. XORed with plane xbit, the last row is
    plane xbit; ``blocks`` > 1: the source holds that many blocks of the output's elements and
    the last ``blocks`` rows are plane xbit of each (bits_party.h plane_of).  Phases 0 / 1
    return state (msg, z, base0, base1);
    phase 2 (state + the received z in ``arecv``) returns the result pair [count, ...]."""
    like = next(t for t in src if t is not None) if src is not None else state[1]
    per = tuple(like.shape[:-1] if bits == 128 else like.shape) if src is not None else None
    if phase == 2:
        msg, z, b0, b1 = state
        S = z.numel() // (2 if bits == 128 else 1) // count
        o0, o1 = torch.empty_like(z), torch.empty_like(z)
        nat.check(nat.lib().mx_bits_b2a(
            nat.dev_of(z), _words(bits), 2, role, S, start, count, xbit, blocks, None, None,
            None, _p(z),
            _p(b0), _p(b1), _p(arecv), _p(o0), _p(o1), _slots_arr(slots), _nonces_arr((n1, ng)),
            nat.stream_of(z)), "bits_b2a")
        return o0, o1
    nb = blocks & 0xff  # bits_party.h plane_of: blocks >> 8 is the tail rows' sign plane
    if nb > 1:  # ``nb`` copies concatenated on axis 0: the rows are one block's
        per = (per[0] // nb,) + per[1:]
    S = math.prod(per)
    shp = (count,) + per + ((2,) if bits == 128 else ())
    b0, b1 = (torch.empty(shp, dtype=torch.int64, device=like.device) for _ in range(2))
    msg = _new(alloc, shp, torch.int64, like.device) if role == 0 else None
    z = _new(alloc, shp, torch.int64, like.device)
    srcs = (ctypes.c_void_p * 6)(*[_p(t) for t in src])
    nat.check(nat.lib().mx_bits_b2a(
        nat.dev_of(like), _words(bits), phase, role, S, start, count, xbit, blocks, srcs,
        _p(arecv),
        _p(msg),
        _p(z), _p(b0), _p(b1), None, None, None, _slots_arr(slots), _nonces_arr((n1, ng)),
        nat.stream_of(like)), "bits_b2a")
    return msg, z, b0, b1


def _ring_words(values, bits):
    """Python ints -> a ctypes int64 array of their little-endian 64-bit words (mod 2^bits)."""
    w = _words(bits)
    out = []
    for v in values:
        v = int(v) % (1 << bits)
        for j in range(w):
            out.append(_to_i64((v >> (64 * j)) & MASK64))
    return (ctypes.c_int64 * max(1, len(out)))(*out)


def wsum_pair(bits, L, rows=None, weights=(), x=None, wx=0, pub=(False, False), cblk=(0,),
              second=None, like=None, lead=False):
    """Per-party fused weighted sums over both share components (csrc/wsum_pair.h):
    s_c = sum_k weights[k] rows_c[k] + wx x_c; returns (o0, o1) of nblk = len(cblk) blocks
    of L elements, block b = s_c + cblk[b] on the public slots ``pub`` (this party's copies
    of x_0), and with ``second`` = (m2, c2) also (q0, q1) = m2 s_c + c2 on those slots.
    ``rows`` = (r0, r1) tensors holding len(weights) rows of L elements, contiguous.
    ``lead``: (q0, q1) is block 0 of the outputs instead -- (o0, o1) of 1 + nblk blocks,
    no concatenation afterwards."""
    ref = like if like is not None else (rows[0] if rows is not None else x[0])
    nrows = len(weights)
    if nrows > 64 or not 1 <= len(cblk) <= 3:
        raise ValueError("wsum_pair: at most 64 rows and 3 blocks")
    dev = ref.device
    tail = (2,) if bits == 128 else ()
    q0 = q1 = None
    if lead:
        if second is None:
            raise ValueError("wsum_pair: lead needs second")
        b0 = torch.empty(((1 + len(cblk)) * L,) + tail, dtype=torch.int64, device=dev)
        b1 = torch.empty_like(b0)
        q0, q1, o0, o1 = b0[:L], b1[:L], b0[L:], b1[L:]
    else:
        o0 = torch.empty((len(cblk) * L,) + tail, dtype=torch.int64, device=dev)
        o1 = torch.empty_like(o0)
    if second is not None and not lead:
        q0 = torch.empty(((L,) + tail), dtype=torch.int64, device=dev)
        q1 = torch.empty_like(q0)
    r = [None, None] if rows is None else [t.contiguous() for t in rows]
    xx = [None, None] if x is None else [t.contiguous() for t in x]
    m2, c2 = second if second is not None else (0, 0)
    nat.check(nat.lib().mx_wsum_pair(
        nat.dev_of(o0), _words(bits), nrows, len(cblk), 1 if second is not None else 0,
        1 if pub[0] else 0, 1 if pub[1] else 0, L, L, _ring_words(weights, bits),
        _ring_words([wx], bits), _ring_words([m2], bits), _ring_words([c2], bits),
        _ring_words(cblk, bits), _p(r[0]), _p(r[1]), _p(xx[0]), _p(xx[1]), _p(o0), _p(o1),
        _p(q0), _p(q1), nat.stream_of(o0)), "wsum_pair")
    if lead:
        return b0, b1
    return (o0, o1) if second is None else (o0, o1, q0, q1)
