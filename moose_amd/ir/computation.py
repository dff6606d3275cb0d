"""Native IR: placements, constants, signatures, operations and computations.

Parity: reference ``moose/src/computation.rs`` -- ``Placement`` (:1557-1626),
``Signature`` (:620-767), ``Operation`` (:1656), ``as_graph`` with send->receive
edges keyed by rendezvous key (:1879-1942), msgpack/bincode serde (:1797-1874).
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass
from dataclasses import field
from typing import Any
from typing import Dict
from typing import List
from typing import Optional
from typing import Tuple

import numpy as np

from moose_amd.ir.types import Ty

# ---------------------------------------------------------------------------
# placements
# ---------------------------------------------------------------------------


@dataclass(frozen=True)
class HostPlacement:
    owner: str

    def to_textual(self):
        return f"@Host({self.owner})"

    @property
    def owners(self):
        return (self.owner,)


@dataclass(frozen=True)
class ReplicatedPlacement:
    owners: Tuple[str, str, str]

    def to_textual(self):
        return f"@Replicated({', '.join(self.owners)})"


@dataclass(frozen=True)
class AdditivePlacement:
    owners: Tuple[str, str]

    def to_textual(self):
        return f"@Additive({', '.join(self.owners)})"


@dataclass(frozen=True)
class Mirrored3Placement:
    owners: Tuple[str, str, str]

    def to_textual(self):
        return f"@Mirrored3({', '.join(self.owners)})"


Placement = Any  # union of the four placement classes

PLACEMENT_KINDS = {
    "Host": HostPlacement,
    "Replicated": ReplicatedPlacement,
    "Additive": AdditivePlacement,
    "Mirrored3": Mirrored3Placement,
}


def placement_from(kind: str, owners):
    owners = tuple(owners)
    if kind == "Host":
        (o,) = owners
        return HostPlacement(o)
    n = {"Replicated": 3, "Mirrored3": 3, "Additive": 2}[kind]
    if len(owners) != n:
        raise ValueError(f"{kind} placement expects {n} owners, found {owners}")
    return PLACEMENT_KINDS[kind](owners)


# ---------------------------------------------------------------------------
# constants (literals embedded in Constant/Fill ops)
# ---------------------------------------------------------------------------
TENSOR_CONSTANT_NP = {
    "HostFloat32Tensor": np.float32,
    "HostFloat64Tensor": np.float64,
    "HostInt8Tensor": np.int8,
    "HostInt16Tensor": np.int16,
    "HostInt32Tensor": np.int32,
    "HostInt64Tensor": np.int64,
    "HostUint8Tensor": np.uint8,
    "HostUint16Tensor": np.uint16,
    "HostUint32Tensor": np.uint32,
    "HostUint64Tensor": np.uint64,
    "HostRing64Tensor": np.uint64,
    "HostRing128Tensor": object,  # python ints
    "HostBitTensor": np.uint8,
}
SCALAR_CONSTANTS = ("Ring64", "Ring128", "Bit", "Float32", "Float64")


@dataclass(frozen=True, eq=False)
class Constant:
    """A typed literal. ``kind`` is the textual constructor name
    (``HostFloat64Tensor``, ``Ring128``, ``HostShape``, ``HostString``...)."""

    kind: str
    value: Any

    def __eq__(self, other):
        if not isinstance(other, Constant) or other.kind != self.kind:
            return False
        a, b = self.value, other.value
        if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
            a, b = np.asarray(a), np.asarray(b)
            return a.shape == b.shape and bool(np.all(a == b))
        return a == b

    def __hash__(self):
        v = self.value
        if isinstance(v, np.ndarray):
            return hash((self.kind, v.shape, v.tobytes() if v.dtype != object else str(v)))
        if isinstance(v, list):
            v = tuple(v)
        return hash((self.kind, v))

    @property
    def ty(self) -> Ty:
        if self.kind == "HostString":
            return Ty("HostString")
        return Ty(self.kind)

    def to_textual(self):
        k, v = self.kind, self.value
        if k in TENSOR_CONSTANT_NP:
            return f"{k}({_array_literal(np.asarray(v), k)})"
        if k == "HostShape":
            return f"HostShape([{', '.join(str(int(d)) for d in v)}])"
        if k == "HostString":
            return f"HostString({_quote(v)})"
        if k in ("HostSeed", "HostPrfKey"):
            return f"{k}({bytes(v).hex()})"
        if k in ("Float32", "Float64"):
            return f"{k}({_float_literal(v)})"
        if k in ("Ring64", "Ring128", "Bit"):
            return f"{k}({int(v)})"
        if k == "Fixed":
            val, i, f = v
            return f"Fixed({_float_literal(val)}, {i}, {f})"
        raise ValueError(f"cannot print constant kind {k}")


def _quote(s: str) -> str:
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'


def _float_literal(x) -> str:
    x = float(x)
    if np.isnan(x):
        return "NaN"
    if np.isinf(x):
        return "inf" if x > 0 else "-inf"
    r = repr(x)
    if "e" in r or "E" in r:
        r = np.format_float_positional(x, trim="0")
        if r.endswith("."):
            r += "0"
    return r


def _array_literal(a: np.ndarray, kind: str) -> str:
    is_float = kind in ("HostFloat32Tensor", "HostFloat64Tensor")

    def scalar(x):
        return _float_literal(x) if is_float else str(int(x))

    def rec(x):
        if x.ndim == 0:
            return scalar(x.item() if hasattr(x, "item") else x)
        if x.ndim == 1:
            return "[" + ", ".join(scalar(e) for e in x.tolist()) + "]"
        return "[" + ", ".join(rec(x[i]) for i in range(x.shape[0])) + "]"

    if a.ndim == 0:
        return "[" + scalar(a.item()) + "]" if False else scalar(a.item())
    return rec(a)


# ---------------------------------------------------------------------------
# signatures and operations
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class Signature:
    args: Tuple[Ty, ...]
    ret: Ty
    variadic: bool = False

    @staticmethod
    def nullary(ret):
        return Signature((), ret)

    @staticmethod
    def unary(a, ret):
        return Signature((a,), ret)

    @staticmethod
    def binary(a, b, ret):
        return Signature((a, b), ret)

    @staticmethod
    def ternary(a, b, c, ret):
        return Signature((a, b, c), ret)

    @staticmethod
    def variadic_of(a, ret):
        return Signature((a,), ret, True)

    def arg(self, i) -> Ty:
        return self.args[0] if self.variadic else self.args[i]

    def to_textual(self):
        if self.variadic:
            return f"[{self.args[0].to_textual()}] -> {self.ret.to_textual()}"
        return f"({', '.join(a.to_textual() for a in self.args)}) -> {self.ret.to_textual()}"


@dataclass
class Operation:
    name: str
    kind: str
    inputs: List[str]
    placement: Placement
    sig: Signature
    attrs: Dict[str, Any] = field(default_factory=dict)

    def to_textual(self):
        from moose_amd.ir.textual import print_operation

        return print_operation(self)


class Computation:
    """An ordered list of operations (the order is a valid schedule after toposort)."""

    def __init__(self, operations: Optional[List[Operation]] = None):
        self.operations: List[Operation] = list(operations or [])

    def __len__(self):
        return len(self.operations)

    def __iter__(self):
        return iter(self.operations)

    def by_name(self) -> Dict[str, Operation]:
        return {op.name: op for op in self.operations}

    def placements(self):
        seen = {}
        for op in self.operations:
            seen.setdefault(op.placement, None)
        return list(seen)

    def roles(self):
        roles = {}
        for op in self.operations:
            for o in op.placement.owners:
                roles.setdefault(o, None)
        return list(roles)

    def with_roles(self, assignment: Dict[str, str]) -> "Computation":
        """Copy with every role renamed to its identity (``role -> identity``; roles not
        in ``assignment`` keep their name) -- the role assignment the reference's
        executors apply when they pick an identity's operations
        (``execution/asynchronous.rs:579-605``).  Send/Receive peers are renamed too."""
        import dataclasses

        def ren(plc):
            if isinstance(plc, HostPlacement):
                return HostPlacement(assignment.get(plc.owner, plc.owner))
            return type(plc)(tuple(assignment.get(o, o) for o in plc.owners))

        ops = []
        for op in self.operations:
            attrs = dict(op.attrs)
            for k in ("sender", "receiver"):
                if isinstance(attrs.get(k), str):
                    attrs[k] = assignment.get(attrs[k], attrs[k])
            ops.append(dataclasses.replace(op, placement=ren(op.placement), attrs=attrs))
        return Computation(ops)

    # textual ---------------------------------------------------------------
    def to_textual(self) -> str:
        from moose_amd.ir.textual import print_computation

        return print_computation(self)

    @staticmethod
    def from_textual(source: str, parallel: bool = True) -> "Computation":
        from moose_amd.ir.textual import parse_computation

        return parse_computation(source, parallel=parallel)

    # msgpack ----------------------------------------------------------------
    def to_msgpack(self) -> bytes:
        from moose_amd.ir.serde import to_msgpack

        return to_msgpack(self)

    @staticmethod
    def from_msgpack(data: bytes) -> "Computation":
        from moose_amd.ir.serde import from_msgpack

        return from_msgpack(data)

    # bincode-style binary (reference computation.rs:1837-1844) -------------------
    def to_bincode(self) -> bytes:
        from moose_amd.ir.bincode import to_bincode

        return to_bincode(self)

    @staticmethod
    def from_bincode(data: bytes) -> "Computation":
        from moose_amd.ir.bincode import from_bincode

        return from_bincode(data)

    def to_disk(self, path):
        with open(path, "wb") as f:
            f.write(self.to_msgpack())

    @staticmethod
    def from_disk(path) -> "Computation":
        with open(path, "rb") as f:
            return Computation.from_msgpack(f.read())

    # graph --------------------------------------------------------------------
    def dependency_edges(self):
        """Yield (src_index, dst_index) edges: data edges plus Send->Receive edges
        matched by rendezvous key (reference computation.rs:1879-1942)."""
        index = {op.name: i for i, op in enumerate(self.operations)}
        sends = {}
        for i, op in enumerate(self.operations):
            if op.kind == "Send":
                sends[bytes(op.attrs["rendezvous_key"])] = i
        for j, op in enumerate(self.operations):
            for inp in op.inputs:
                if inp not in index:
                    raise KeyError(f"operation {op.name} refers to unknown input {inp}")
                yield index[inp], j
            if op.kind == "Receive":
                k = bytes(op.attrs["rendezvous_key"])
                if k in sends:
                    yield sends[k], j

    def toposorted(self) -> "Computation":
        from moose_amd.runtime import native_rt

        if native_rt.enabled():
            try:
                return native_rt.toposort(self)
            except native_rt.mod().NativeGraphError as e:
                msg = str(e)
                if "unknown input" in msg:
                    raise KeyError(msg) from None
                raise ValueError(msg) from None
        return self.toposorted_py()

    def toposorted_py(self) -> "Computation":
        n = len(self.operations)
        succ = [[] for _ in range(n)]
        indeg = [0] * n
        for a, b in self.dependency_edges():
            succ[a].append(b)
            indeg[b] += 1
        ready = [i for i in range(n) if indeg[i] == 0]
        ready.reverse()
        order = []
        while ready:
            i = ready.pop()
            order.append(i)
            for j in reversed(succ[i]):
                indeg[j] -= 1
                if indeg[j] == 0:
                    ready.append(j)
        if len(order) != n:
            raise ValueError("computation graph has a cycle")
        return Computation([self.operations[i] for i in order])

    def digest(self) -> str:
        """Stable content hash (used as the compiled-plan cache key)."""
        return hashlib.blake2b(self.to_textual().encode(), digest_size=16).hexdigest()


# ---------------------------------------------------------------------------
# session ids and rendezvous keys
# ---------------------------------------------------------------------------
class SessionId:
    """16-byte session identifier derived from a logical name (blake2b stands in
    for the reference's blake3, computation.rs:96-144)."""

    def __init__(self, logical: str):
        self.logical = logical
        self.secure = hashlib.blake2b(logical.encode(), digest_size=16).digest()

    @staticmethod
    def random() -> "SessionId":
        return SessionId(os.urandom(16).hex())

    def __repr__(self):
        return f"SessionId({self.logical!r})"

    def __eq__(self, other):
        return isinstance(other, SessionId) and other.secure == self.secure

    def __hash__(self):
        return hash(self.secure)


def rendezvous_key_from_counter(n: int) -> bytes:
    return int(n).to_bytes(16, "little")
