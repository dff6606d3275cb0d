"""Host-level primitive operations (the leaf kernels of a lowered graph).

Each primitive has a name -- the operator kind it becomes in a lowered computation
(``Add``, ``Dot``, ``SampleSeeded`` ... and this framework's fused extensions
``RingMulCross``/``RingDotCross``/``BitAndCross``/``ZeroShare``) -- an eager
implementation on python/torch values, and a result-type rule used by the symbolic
session.  Eager values are:

* :class:`moose_amd.ops.ring.RT` for ring / bit tensors,
* ``torch.Tensor`` for plaintext host tensors (float, int, uint, bool),
* ``tuple`` for shapes, ``bytes`` for PRF keys / seeds, ``str`` for strings.

Implementations take ``nb`` -- the number of leading batch dims (1 when the three
parties of a session are stacked on one device) -- so axis attributes stay logical.

Parity: the ``runtime`` flavour rows of the reference dispatch tables
(``moose/src/kernels/*.rs``) are the host kernels in ``moose/src/host/ops.rs``.
"""
from __future__ import annotations

import math

import torch

from moose_amd.ir import types as T
from moose_amd.ops import ring as R


class Prim:
    __slots__ = ("name", "impl", "ty")

    def __init__(self, name, impl, ty=None):
        self.name = name
        self.impl = impl
        self.ty = ty or (lambda tys, **a: tys[0])


PRIMS = {}


def prim(name, ty=None):
    def deco(fn):
        PRIMS[name] = Prim(name, fn, ty)
        return fn

    return deco


def _is_rt(x):
    return isinstance(x, R.RT)


def _tensorish(x):
    return isinstance(x, (R.RT, torch.Tensor))


# ---------------------------------------------------------------------------
# arithmetic (ring or plaintext)
# ---------------------------------------------------------------------------
def _arith(op):
    def impl(nb, a, b):
        if _is_rt(a) or _is_rt(b):
            return R.binary(op, a, b)
        if op == "add":
            return a + b
        if op == "sub":
            return a - b
        if op == "mul":
            return a * b
        if op == "and":
            return a & b
        if op == "or":
            return a | b
        if op == "xor":
            return a ^ b
        raise AssertionError(op)

    return impl


prim("Add")(_arith("add"))
prim("Sub")(_arith("sub"))
prim("Mul")(_arith("mul"))
prim("And")(_arith("and"))
prim("Or")(_arith("or"))
prim("Xor")(_arith("xor"))


@prim("MulLeading")
def _mul_leading(nb, a, c):
    """a[..., i, ...] * c[i] along the first non-party axis of ``a`` (``c`` 1-D public):
    a rank-agnostic scaling, so shape-polymorphic lowering can express it."""
    if not _is_rt(a):
        k = a.dim() - nb - 1
        return a * c.reshape((c.shape[0],) + (1,) * k)
    return R.mul_leading(a, c, nb)


@prim("Neg")
def _neg(nb, a):
    if _is_rt(a):  # on bit tensors Neg is NOT (reference host/ops.rs:1519-1527)
        return ~a if a.bits == 1 else -a
    if a.dtype == torch.bool:
        return ~a
    return -a


@prim("Div")
def _div(nb, a, b):
    if _is_rt(a):
        return _ring_div(a, b)
    if a.dtype in (torch.float32, torch.float64):
        return a / b
    return torch.div(a, b, rounding_mode="trunc")


def _ring_div(a, b):
    """Unsigned integer division of ring tensors (``Wrapping<u64> / Wrapping<u128>``,
    reference host/ops.rs:334-343).  A host-only kernel on python integers: no protocol
    divides ring values, so it is never on a hot path."""
    import numpy as np

    x, y = R.to_ints(a), R.to_ints(b)
    x, y = np.broadcast_arrays(x, y)
    if any(int(v) == 0 for v in y.reshape(-1)):
        raise ZeroDivisionError("ring division by zero")
    q = np.vectorize(lambda u, v: int(u) // int(v), otypes=[object])(x, y)
    return R.from_ints(q, a.bits, a.device)


@prim("Shl")
def _shl(nb, a, amount):
    return a.shl(amount)


@prim("Shr")
def _shr(nb, a, amount):
    return a.shr(amount)


@prim("Sar")
def _sar(nb, a, amount):
    return a.sar(amount)


@prim("Dot")
def _dot(nb, a, b):
    if _is_rt(a):
        return R.dot(a, b, nb)
    if nb:
        return torch.matmul(a, b)
    if a.dim() <= 2 and b.dim() <= 2:
        return a @ b if (a.dim() > 0 and b.dim() > 0) else a * b
    return torch.tensordot(a, b, dims=([a.dim() - 1], [0]))


@prim("Sum", ty=lambda tys, **a: tys[0])
def _sum(nb, a, axis=None):
    if _is_rt(a):
        return R.sum(a, axis, nb)
    if axis is None:
        return a.reshape(a.shape[:nb] + (-1,)).sum(dim=nb) if nb else a.sum()
    return a.sum(dim=_lax(a.dim(), axis, nb))


def _lax(ndim, axis, nb):
    nd = ndim - nb
    return (axis + nd if axis < 0 else axis) + nb


@prim("AddN")
def _addn(nb, *xs):
    acc = xs[0]
    for x in xs[1:]:
        acc = _arith("add")(nb, acc, x)
    return acc


@prim("Mean")
def _mean(nb, a, axis=None):
    if axis is None:
        return a.mean() if not nb else a.reshape(a.shape[:nb] + (-1,)).mean(dim=nb)
    return a.mean(dim=_lax(a.dim(), axis, nb))


@prim("RingFixedpointMean")
def _ring_fixedpoint_mean(nb, a, axis=None, scaling_base=2, scaling_exp=0):
    """Sum along ``axis`` (all entries when None) times the mean weight 1/n encoded with
    scaling_base^scaling_exp -- the float product truncated toward zero, as the
    reference's encode (host/fixedpoint.rs:66-76, 10-38).  No truncation of the product:
    the result carries twice the fractional bits, as the reference's."""
    shape = a.shape[nb:]
    n = shape[axis] if axis is not None else math.prod(shape)
    w = int((1.0 / n) * float(int(scaling_base) ** int(scaling_exp)))
    s = R.sum(a, axis, nb)
    return R.binary("mul", s, R.fill((), w % (1 << a.bits), a.bits, a.device))


@prim("RingFixedpointArgmax", ty=lambda tys, **a: T.Ty("HostRing64Tensor"))
def _ring_fixedpoint_argmax(nb, a, axis, upmost_index=None):
    """Index of the first maximum along ``axis``, entries read as signed ring values; a
    Z_2^64 tensor of indices (reference host/ops.rs:2374-2445)."""
    ax = _lax(a.ndim, axis, nb)
    d = a.data
    n = d.shape[ax]
    hi = d.select(ax, 0)
    lo = None
    if a.bits == 128:  # (lo, hi) words: signed high word, unsigned low word
        lo = hi[..., 0] ^ _SIGN64
        hi = hi[..., 1]
    best_hi, best_lo = hi.clone(), None if lo is None else lo.clone()
    idx = torch.zeros(best_hi.shape, dtype=torch.int64, device=d.device)
    for i in range(1, n):
        v = d.select(ax, i)
        if a.bits == 128:
            vl, vh = v[..., 0] ^ _SIGN64, v[..., 1]
            gt = (vh > best_hi) | ((vh == best_hi) & (vl > best_lo))
            best_lo = torch.where(gt, vl, best_lo)
        else:
            vh = v
            gt = vh > best_hi
        best_hi = torch.where(gt, vh, best_hi)
        idx = torch.where(gt, torch.full_like(idx, i), idx)
    return R.RT(idx.contiguous(), 64)


_SIGN64 = -(1 << 63)


# ---------------------------------------------------------------------------
# shapes
# ---------------------------------------------------------------------------
@prim("Shape", ty=lambda tys, **a: T.HOST_SHAPE)
def _shape(nb, a):
    if _is_rt(a):
        return tuple(a.shape[nb:])
    return tuple(a.shape[nb:])


@prim("Reshape")
def _reshape(nb, a, shape=None):
    if _is_rt(a):
        return R.reshape(a, shape, nb)
    return a.reshape(tuple(a.shape[:nb]) + tuple(shape))


@prim("ExpandDims")
def _expand_dims(nb, a, axis):
    if _is_rt(a):
        return R.expand_dims(a, axis, nb)
    d = a
    nd = a.dim() - nb
    for ax in sorted(axis):
        if ax < 0:
            ax += nd + 1
        d = d.unsqueeze(ax + nb)
        nd += 1
    return d


@prim("Squeeze")
def _squeeze(nb, a, axis=None):
    if _is_rt(a):
        return R.squeeze(a, axis, nb)
    if axis is None:
        keep = list(a.shape[:nb]) + [s for s in a.shape[nb:] if s != 1]
        return a.reshape(keep)
    return a.squeeze(_lax(a.dim(), axis, nb))


@prim("Transpose")
def _transpose(nb, a):
    if _is_rt(a):
        return R.transpose(a, nb)
    nd = a.dim() - nb
    perm = list(range(nb)) + [nb + i for i in reversed(range(nd))]
    return a.permute(perm).contiguous()


@prim("Concat")
def _concat(nb, *xs, axis=0):
    if _is_rt(xs[0]):
        return R.concat(xs, axis, nb)
    return torch.cat(xs, dim=_lax(xs[0].dim(), axis, nb))


@prim("IndexAxis")
def _index_axis(nb, a, axis, index):
    if _is_rt(a):
        return R.index_axis(a, axis, index, nb)
    return a.select(_lax(a.dim(), axis, nb), index).contiguous()


@prim("Slice")
def _slice(nb, a, slice):
    start, end, step = slice
    if isinstance(a, tuple):  # a shape (HostShape slice, reference host/ops.rs Slice)
        return a[start:end:step]
    if _is_rt(a):
        return R.slice_axis(a, 0, start, end, step, nb)
    idx = [builtins_slice(None)] * nb + [builtins_slice(start, end, step)]
    return a[tuple(idx)].contiguous()


builtins_slice = slice


@prim("Permute")
def _permute(nb, a, perm):
    if _is_rt(a):
        return R.transpose(a, nb, perm)
    return a.permute(list(range(nb)) + [p + nb for p in perm]).contiguous()


@prim("StridedSlice")
def _strided_slice(nb, a, slices):
    if _is_rt(a):
        return R.strided_slice(a, slices, nb)
    idx = [builtins_slice(None)] * nb + list(slices)
    return a[tuple(idx)].contiguous()


@prim("Select")
def _select(nb, a, mask, axis):
    # session primitive order (x, index); the IR op is (index, x) (graph_executor swaps)
    m = mask.data if _is_rt(mask) else mask
    if _is_rt(a):
        return R.select_mask(a, axis, m, nb)
    keep = torch.nonzero(m.reshape(-1).to(torch.bool)).reshape(-1).to(a.device)
    return a.index_select(_lax(a.dim(), axis, nb), keep).contiguous()


@prim("Diag")
def _diag(nb, a):
    if _is_rt(a):
        return R.diag(a, nb)
    return torch.diagonal(a, dim1=nb, dim2=nb + 1).contiguous()


@prim("Broadcast")
def _broadcast(nb, a, shape=None):
    if _is_rt(a):
        return R.broadcast_to(a, shape, nb)
    lead = len(shape) - (a.dim() - nb)
    if lead > 0:
        a = a.reshape(tuple(a.shape[:nb]) + (1,) * lead + tuple(a.shape[nb:]))
    return a.expand(tuple(a.shape[:nb]) + tuple(shape)).contiguous()


@prim("BroadcastLike")
def _broadcast_like(nb, a, like):
    """Broadcast ``a`` to the (run-time) shape of ``like`` -- the shape-polymorphic form of
    Broadcast, for lowered graphs whose shapes are only known when they run."""
    return _broadcast(nb, a, tuple(like.shape[nb:]))


@prim("AtLeast2D")
def _atleast_2d(nb, a, to_column_vector=False):
    if _is_rt(a):
        return R.atleast_2d(a, to_column_vector, nb)
    nd = a.dim() - nb
    if nd >= 2:
        return a
    if nd == 0:
        return a.reshape(tuple(a.shape[:nb]) + (1, 1))
    n = a.shape[nb]
    return a.reshape(tuple(a.shape[:nb]) + ((n, 1) if to_column_vector else (1, n)))


# ---------------------------------------------------------------------------
# constants / randomness
# ---------------------------------------------------------------------------
@prim("Fill")
def _fill(nb, shape, value, bits, device="cpu"):
    return R.fill(shape, value, bits, device)


@prim("AddConst")
def _add_const(nb, x, value, bits):
    """x + value (mod 2^bits); lowers to Fill + Add."""
    return R.binary("add", x, R.fill((), int(value), bits, x.device))


@prim("SampleSeeded")
def _sample_seeded(nb, shape, seed, bits, device="cpu"):
    """Uniform ring tensor expanded from a 16-byte seed: the PRF stream (ChaCha12,
    csrc/prf_core.h) keyed by the seed, nonce 0 (reference ``host/ops.rs:1883-2036`` +
    ``host/prim.rs:123-150``)."""
    if hasattr(seed, "table"):  # a KeyRef: the seed lives in a device key slot
        out = R.prf_expand_k(seed.ptr, 1, 0, tuple(shape), bits, device)
        return R.RT(out.data[0], bits)
    out = R.prf_expand([bytes(seed)[:16]], 0, tuple(shape), bits, device)
    return R.RT(out.data[0], bits)


@prim("DeriveSeed")
def _derive_seed(nb, key, sync_key):
    """16-byte seed = PRF(key) at the 128-bit input given by the sync key (reference
    ``host/prim.rs`` DeriveSeed: a keyed derivation of the sync key; parity of the bytes
    unpinned -- the reference hashes with its own KDF).  Sync keys longer than 16 bytes are
    compressed with BLAKE2b first."""
    import ctypes
    import hashlib

    sk = bytes(sync_key)
    sk = hashlib.blake2b(sk, digest_size=16).digest() if len(sk) > 16 else sk.ljust(16, b"\0")
    out = ctypes.create_string_buffer(16)
    from moose_amd.ops import native as nat

    nat.check(nat.lib().mx_derive_seed(bytes(key)[:16], sk, out), "derive_seed")
    return out.raw


@prim("PrfKeyGen")
def _prf_key_gen(nb):
    import os

    return os.urandom(16)


@prim("Sample")
def _sample(nb, shape, bits, device="cpu"):
    import os

    return _sample_seeded(nb, shape, os.urandom(16), bits, device)


@prim("Zeros")
def _zeros(nb, shape, dtype=torch.float64, device="cpu"):
    return torch.zeros(tuple(shape), dtype=dtype, device=device)


@prim("Ones")
def _ones(nb, shape, dtype=torch.float64, device="cpu"):
    return torch.ones(tuple(shape), dtype=dtype, device=device)


# ---------------------------------------------------------------------------
# ring <-> plaintext
# ---------------------------------------------------------------------------
@prim("RingFixedpointEncode")
def _encode(nb, x, scaling_exp, bits):
    # deferred: an input sharing of the result encodes inside the share kernel
    return R.encode_lazy(x, scaling_exp, bits)


@prim("RingFixedpointDecode")
def _decode(nb, x, scaling_exp, dtype=None):
    out = R.decode(x, scaling_exp)
    return out if dtype is None or out.dtype == dtype else out.to(dtype)


@prim("BitExtract")
def _bit_extract(nb, x, bit_idx):
    return R.bit_extract(x, bit_idx)


@prim("RingInject")
def _ring_inject(nb, x, bit_idx, bits):
    return R.ring_inject(x, bit_idx, bits)


@prim("RingCast")
def _ring_cast(nb, x, bits):
    return R.cast(x, bits)


@prim("BitSplit")
def _bit_split(nb, x, start, count):
    """Packed word -> bit tensor with a new logical leading axis: out[j] = bit start+j."""
    return R.bit_planes(x, start, count, nb)


@prim("WeightedSum")
def _weighted_sum(nb, x, weights, bits):
    """sum_j weights[j] * x[j] over the leading logical axis (public integer weights)."""
    return R.weighted_sum(x, weights, nb)


@prim("BitDecompose")
def _bit_decompose(nb, x, to_bits=True):
    """Ring tensor -> its bits stacked on a new leading logical axis (LSB first), as a
    bit tensor or as 0/1 ring elements (reference host/ops.rs:855-937)."""
    out = R.bit_planes(x, 0, x.bits, nb)
    if to_bits:
        return out
    return R.ring_inject(out, 0, x.bits)


@prim("ShlDim")
def _shl_dim(nb, x, amount, bit_length):
    """Shift along the leading (bit) axis: out[i] = x[i - amount], zeros below
    (reference host/ops.rs:835-853)."""
    d = x.data if _is_rt(x) else x
    ax = nb
    head = torch.zeros_like(d.narrow(ax, 0, amount))
    out = torch.cat([head, d.narrow(ax, 0, bit_length - amount)], dim=ax)
    return R.RT(out, x.bits) if _is_rt(x) else out


@prim("BitAffine")
def _bit_affine(nb, x, aff):
    """Linear part of a GF(2) affine map over the leading logical axis of a bit tensor
    (``aff`` is a ``bristol._SparseAffine``; one sparse GEMM, see protocols/bristol)."""
    d = x.data
    if nb:
        d = d.movedim(0, 1)  # party axis behind the wire axis
    y = aff.linear(d)
    if nb:
        y = y.movedim(1, 0)
    return R.RT(y.contiguous(), 1)


@prim("ToBool")
def _to_bool(nb, x):
    return x.data.to(torch.bool) if _is_rt(x) else x.to(torch.bool)


@prim("FromBool")
def _from_bool(nb, x):
    if _is_rt(x):  # already a bit tensor (e.g. a host comparison result)
        return R.RT(x.data.to(torch.uint8), 1)
    return R.RT(x.to(torch.uint8), 1)


@prim("RingToInt")
def _ring_to_int(nb, x):
    return R.cast(x, 64).data


@prim("IntToRing")
def _int_to_ring(nb, x):
    return R.RT(x.to(torch.int64), 64)


@prim("Less")
def _less(nb, a, b):
    if _is_rt(a):
        return R.compare("lt", a, b)
    return a < b


@prim("Greater")
def _greater(nb, a, b):
    if _is_rt(a):
        return R.compare("gt", a, b)
    return a > b


@prim("Equal")
def _equal(nb, a, b):
    if _is_rt(a):
        return R.compare("eq", a, b)
    return a == b


@prim("Msb")
def _msb(nb, a):
    return R.compare("msb", a)


@prim("Mux")
def _mux(nb, s, x, y):
    if _is_rt(s) and not _is_rt(x):  # a bit selector over plaintext operands
        s = s.data
    if _is_rt(x):
        sel = s if _is_rt(s) else R.RT(s.to(torch.uint8), 1)
        m = R.ring_inject(sel, 0, x.bits) if sel.bits == 1 else sel
        return R.binary("add", R.binary("mul", m, R.binary("sub", x, y)), y)
    return torch.where(s.to(torch.bool), x, y)


# ---------------------------------------------------------------------------
# plaintext float math (host placements)
# ---------------------------------------------------------------------------
def _f(fn):
    def impl(nb, a, **kw):
        return fn(a, **kw)

    return impl


prim("Exp")(_f(torch.exp))
prim("Log")(_f(torch.log))
prim("Log2")(_f(torch.log2))
prim("Sqrt")(_f(torch.sqrt))
prim("Sigmoid")(_f(torch.sigmoid))
prim("Relu")(_f(torch.relu))
prim("Abs")(_f(torch.abs))
@prim("Sign")
def _sign(nb, a):
    """Plaintext: torch.sign.  Ring: -1 for negative (two's complement) entries, +1
    otherwise -- zero included (reference host/ops.rs:1420-1452)."""
    if not _is_rt(a):
        return torch.sign(a)
    d = a.data if a.bits == 64 else a.data[..., 1]
    neg = d < 0
    if a.bits == 64:
        return R.RT(torch.where(neg, -1, 1).to(torch.int64), 64)
    lo = torch.where(neg, -1, 1).to(torch.int64)
    hi = torch.where(neg, -1, 0).to(torch.int64)
    return R.RT(torch.stack([lo, hi], dim=-1), 128)
def _inverse(a):
    """torch.linalg.inv without its error check on device tensors: the check reads the
    solver's info flag back to the host, which a hipGraph capture cannot do (a singular
    input gives inf/nan entries instead of an exception, like numpy's LinAlgError-free
    paths; on the host the checked form runs)."""
    if a.is_cuda:
        return torch.linalg.inv_ex(a)[0]
    return torch.linalg.inv(a)


prim("Inverse")(_f(_inverse))


@prim("Softmax")
def _softmax(nb, a, axis, upmost_index):
    ax = _lax(a.dim(), axis, nb)
    return torch.softmax(a, dim=ax)


@prim("Argmax", ty=lambda tys, **a: T.Ty("HostUint64Tensor"))
def _argmax(nb, a, axis, upmost_index):
    ax = _lax(a.dim(), axis, nb)
    return torch.argmax(a, dim=ax)


@prim("Maximum")
def _maximum(nb, *xs):
    if _is_rt(xs[0]):
        return _ring_maximum(xs)
    acc = xs[0]
    for x in xs[1:]:
        acc = torch.maximum(acc, x)
    return acc


def _ring_maximum(xs):
    """Elementwise maximum of ring tensors compared as UNSIGNED integers -- the reference's
    ring Maximum compares ``Wrapping<u64>`` / ``Wrapping<u128>`` (host/ops.rs:2475-2497)."""
    bits = xs[0].bits
    acc = xs[0].data
    for x in xs[1:]:
        d = x.data
        if bits == 128:
            ah, bh = acc[..., 1] ^ _SIGN64, d[..., 1] ^ _SIGN64
            al, bl = acc[..., 0] ^ _SIGN64, d[..., 0] ^ _SIGN64
            gt = (bh > ah) | ((bh == ah) & (bl > al))
            acc = torch.where(gt.unsqueeze(-1), d, acc)
        elif bits == 64:
            acc = torch.where((d ^ _SIGN64) > (acc ^ _SIGN64), d, acc)
        else:
            acc = torch.maximum(acc, d)
    return R.RT(acc.contiguous(), bits)


@prim("Cast")
def _cast(nb, x, dtype=torch.float64, ty=None):
    """Host casts (reference kernels/conversion.rs:26-48).  ``ty`` is the result type name
    when known (a lowered graph): rings and bits need it."""
    if ty == "HostBitTensor":  # x != 0 (host/ops.rs:2334-2371)
        d = x.data if _is_rt(x) else x
        return R.RT((d != 0).to(torch.uint8), 1)
    if ty in ("HostRing64Tensor", "HostRing128Tensor"):
        bits = 64 if ty == "HostRing64Tensor" else 128
        return x if x.bits == bits else R.cast(x, bits)
    if _is_rt(x):  # bit -> float / u64 (0 / 1); Z_2^64 -> u64 (the same 64 bits)
        return x.data.to(dtype)
    return x.to(dtype)


@prim("Identity")
def _identity(nb, x):
    return x


def numel_of(shape):
    return math.prod(shape)
