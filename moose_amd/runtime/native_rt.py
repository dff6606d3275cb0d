"""Python face of the native runtime core (``csrc/runtime``, extension ``_moosert``).

The C++ core holds the parts of the reference's Rust runtime that are not tensor math:

* the textual parser (reference ``textual/parsing.rs``; chunks parsed on native threads);
* the graph (``computation.rs:1879-1942`` ``as_graph``, ``compilation/toposort.rs``,
  ``pruning.rs``, ``well_formed.rs``) used by every pass and executor;
* the dataflow scheduler (``execution/asynchronous.rs``: every op runs once its operands
  are ready, receives wait on the network, the first error aborts the session);
* networking (``networking/local.rs`` single-assignment rendezvous cells and
  ``networking/tcpstream.rs`` length-framed TCP with per-peer send threads and backoff).

``MOOSEX_NATIVE_RUNTIME=0`` selects the pure-Python implementations (kept as the
oracle the native paths are tested against).
"""
from __future__ import annotations

import functools
import os
import threading

import numpy as np

_MOD = None
_LOCK = threading.Lock()


def mod():
    """The loaded extension; built in-tree on first use when sources are newer."""
    global _MOD
    if _MOD is None:
        with _LOCK:
            if _MOD is None:
                from moose_amd._native import build as _build

                if _build.runtime_needs_build():
                    _build.build_runtime()
                from moose_amd._native import _moosert

                _MOD = _moosert
    return _MOD


def enabled() -> bool:
    if os.environ.get("MOOSEX_NATIVE_RUNTIME", "1") == "0":
        return False
    try:
        mod()
        return True
    except Exception:  # no compiler and no prebuilt extension
        return False


@functools.lru_cache(maxsize=1)
def schema():
    from moose_amd.ir.operators import ALL_OPERATORS
    from moose_amd.ir.operators import DEFAULT_RETURN
    from moose_amd.ir.operators import OPERATOR_ALIASES

    ops = {k: [tuple(a) for a in v] for k, v in ALL_OPERATORS.items()}
    return mod().Schema(ops, dict(OPERATOR_ALIASES), dict(DEFAULT_RETURN))


@functools.lru_cache(maxsize=8192)
def _ty(txt):
    from moose_amd.ir.types import Ty

    return Ty.from_textual(txt)


@functools.lru_cache(maxsize=4096)
def _placement(kind, owners):
    from moose_amd.ir.computation import placement_from

    return placement_from(kind, owners)


def _constant(v):
    from moose_amd.ir.computation import Constant
    from moose_amd.ir.computation import TENSOR_CONSTANT_NP

    kind = v[1]
    if kind in TENSOR_CONSTANT_NP:
        flat, shape = v[2], tuple(v[3])
        npd = TENSOR_CONSTANT_NP[kind]
        arr = np.array(flat, dtype=object if npd is object else npd)
        return Constant(kind, arr.reshape(shape))
    if kind == "HostShape":
        return Constant(kind, tuple(int(x) for x in v[2]))
    if kind in ("HostString", "HostSeed", "HostPrfKey"):
        return Constant(kind, v[2])
    if kind in ("Ring64", "Ring128", "Bit"):
        return Constant(kind, int(v[2][0]))
    if kind in ("Float32", "Float64"):
        return Constant(kind, float(v[2][0]))
    if kind == "Fixed":
        val, i, f = v[2]
        return Constant("Fixed", (float(val), int(i), int(f)))
    raise ValueError(f"unknown constant kind {kind}")


def _attr(v):
    if isinstance(v, tuple) and v and v[0] == "const":
        return _constant(v)
    return v


def parse(source: str, threads: int = 8):
    """Textual source -> :class:`~moose_amd.ir.computation.Computation`."""
    from moose_amd.ir.computation import Computation
    from moose_amd.ir.computation import Operation
    from moose_amd.ir.computation import Signature
    from moose_amd.ir.types import Ty

    recs = mod().parse(source, schema(), threads)
    ops = []
    for name, kind, attrs, sig, sig_default, inputs, pk, owners in recs:
        if sig is None:
            signature = Signature((), Ty(sig_default))
        else:
            args, ret, variadic = sig
            signature = Signature(tuple(_ty(t) for t in args), _ty(ret), variadic)
        try:
            plc = _placement(pk, tuple(owners))
        except (KeyError, ValueError) as e:
            raise ValueError(f"{name}: {e}") from None
        ops.append(Operation(name, kind, inputs, plc, signature,
                             {k: _attr(x) for k, x in attrs}))
    return Computation(ops)


def rdv_hex(op) -> str:
    return bytes(op.attrs["rendezvous_key"]).hex()


def graph_of(comp):
    """Native :class:`Graph` of a computation (data edges + Send->Receive edges)."""
    ops = comp.operations
    names = [op.name for op in ops]
    inputs = [list(op.inputs) for op in ops]
    kinds = [op.kind for op in ops]
    rdv = [rdv_hex(op) if op.kind in ("Send", "Receive") else "" for op in ops]
    hosts = [getattr(op.placement, "owner", "") for op in ops]
    return mod().Graph(names, inputs, kinds, rdv, hosts)


def toposort(comp):
    from moose_amd.ir.computation import Computation

    order = graph_of(comp).toposort()
    ops = comp.operations
    return Computation([ops[i] for i in order])


def prune(comp):
    from moose_amd.ir.computation import Computation

    keep = graph_of(comp).prune()
    ops = comp.operations
    return Computation([ops[i] for i in keep])


def stats(comp) -> dict:
    """Static graph metrics (the reference's ``elk stats`` plus depth / comm rounds)."""
    g = graph_of(comp)
    lv = g.levels()
    return {
        "ops": len(g),
        "op_histogram": dict(g.op_histogram()),
        "out_degree": dict(g.out_degree_histogram()),
        "depth": (max(lv) + 1) if lv else 0,
        "comm_rounds": g.comm_rounds(),
    }
