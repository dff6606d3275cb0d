"""Share IO: pre-shared replicated inputs and per-party share checkpoints.

* **Pre-shared inputs** (reference ``moose/src/replicated/input.rs:11-104``): an ``Input``
  op on a replicated placement whose type is ``Replicated{Ring64,Ring128,Bit,Fixed64,
  Fixed128}Tensor`` / ``ReplicatedBitArray{64,128,224}`` reads, for party *i* with role
  ``r_i``, the two arguments ``"{arg}/{r_i}/share{i}"`` and ``"{arg}/{r_i}/share{i+1}"``
  -- the party's pair ``[x_i, x_{i+1}]`` of the RSS layout
  ``[[x00,x10],[x11,x21],[x22,x02]]``.  Fixed-point precisions follow the reference:
  ``(14, 23)`` for Fixed64 and ``(24, 40)`` for Fixed128 unless the op's logical type
  names them.
* **Share checkpoints** (SURVEY §5 "checkpoint / resume"): ``Save`` on a replicated
  placement stores each party's two shares in *that party's own* storage under the same
  ``"{key}/{role}/share{i}"`` names (plus a ``"{key}/{role}/meta"`` JSON string with ring
  width, kind and precision), so nothing secret is ever combined; ``Load`` on a
  replicated placement reassembles the sharing from the parties' storages.  A training
  loop can therefore stop and resume from secret-shared weights without revealing them.

Host encoding of one share: Z_2^64 -> ``uint64[...]``; Z_2^128 -> ``uint64[..., 2]``
(little-endian limbs, lo then hi); bits -> ``uint8[...]``.
"""
from __future__ import annotations

import json
from typing import Callable
from typing import Optional

import numpy as np
import torch

from moose_amd.ir import types as T
from moose_amd.ops import ring as R
from moose_amd.runtime.session import HV

# replicated Input/Load return types -> (ring bits, kind, default fixed dtype)
REP_TYPES = {
    "ReplicatedRing64Tensor": (64, "arith", None),
    "ReplicatedRing128Tensor": (128, "arith", None),
    "ReplicatedBitTensor": (1, "bool", None),
    "ReplicatedFixed64Tensor": (64, "arith", T.fixed64(14, 23)),
    "ReplicatedFixed128Tensor": (128, "arith", T.fixed128(24, 40)),
    "ReplicatedBitArray64": (1, "bool", None),
    "ReplicatedBitArray128": (1, "bool", None),
    "ReplicatedBitArray224": (1, "bool", None),
}


def share_name(key: str, role: str, i: int) -> str:
    return f"{key}/{role}/share{i}"


def meta_name(key: str, role: str) -> str:
    return f"{key}/{role}/meta"


def ring_from_python(value, bits: int, device) -> R.RT:
    """One share from its host encoding (also accepts RT / torch tensors / int lists)."""
    if isinstance(value, R.RT):
        if value.bits != bits:
            raise TypeError(f"share is Z_2^{value.bits}, expected Z_2^{bits}")
        return R.RT(R.to_device(value.data, device), bits)
    if isinstance(value, torch.Tensor):
        return R.RT(R.to_device(value, device), bits)
    a = np.asarray(value)
    if a.dtype == object:
        return R.from_ints(a.tolist(), bits, device)
    if bits == 1:
        return R.RT(R.to_device(torch.from_numpy(np.ascontiguousarray(a.astype(np.uint8))),
                                device), 1)
    if a.dtype.kind not in "iu":
        raise TypeError(f"ring shares must be integer arrays, got {a.dtype}")
    a = np.ascontiguousarray(a.astype(np.uint64, copy=False)).view(np.int64)
    if bits == 128 and (a.ndim == 0 or a.shape[-1] != 2):
        raise ValueError("a Z_2^128 share is a uint64[..., 2] (lo, hi) array")
    return R.RT(R.to_device(torch.from_numpy(a.copy()), device), bits)


def ring_to_python(x: R.RT) -> np.ndarray:
    d = x.data.detach().cpu()
    if x.bits == 1:
        return d.numpy().astype(np.uint8)
    return d.numpy().view(np.uint64).copy()


def rep_from_components(sess, plc, bits, kind, lookup: Callable[[int, int], object]):
    """RepTensor from each party's own pair of shares; ``lookup(party, share_index)``
    returns the host encoding (only called for parties this process holds)."""
    from moose_amd.parallel.spmd import Remote
    from moose_amd.protocols.replicated import RepTensor

    me = getattr(sess, "me", None)
    o = plc.owners
    c0, c1 = [], []
    for p in range(3):
        if me is not None and me != o[p]:
            c0.append(HV(o[p], Remote(bits)))
            c1.append(HV(o[p], Remote(bits)))
            continue
        c0.append(HV(o[p], ring_from_python(lookup(p, p), bits, sess.device)))
        c1.append(HV(o[p], ring_from_python(lookup(p, (p + 1) % 3), bits, sess.device)))
    return RepTensor(plc, bits, kind, sess.gather(plc, c0), sess.gather(plc, c1))


def rep_components(sess, t):
    """Per party i: ``(x_i, x_{i+1})`` host values (``None`` where not held here)."""
    out = []
    for p in range(3):
        a, b = sess.take(t.s0, p), sess.take(t.s1, p)
        if not (sess.materialized(a) and sess.materialized(b)):
            out.append(None)
        else:
            out.append((a.v, b.v))
    return out


def meta_json(bits, kind, dtype: Optional[T.TensorDType]) -> str:
    m = {"bits": bits, "kind": kind}
    if dtype is not None:
        m["dtype"] = dtype.to_textual()
    return json.dumps(m)


def parse_meta(s) -> dict:
    m = json.loads(s if isinstance(s, str) else str(s))
    if "dtype" in m:
        m["dtype"] = T.TensorDType.from_textual(m["dtype"])
    return m
