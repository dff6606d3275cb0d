"""Compiler passes and driver (the ``elk`` compiler).

Parity with the reference ``moose/src/compilation``:

==================  =============================================  ===================
pass name           reference                                      here
==================  =============================================  ===================
``typing``          typing.rs:7-257 (one-hop signature merge)      :func:`typing_pass`
``deprecatedShape`` deprecated_shape.rs:5-43                       :func:`deprecated_shape`
``lowering``        lowering.rs + execution/symbolic.rs:400-435    :func:`lowering`
``prune``           pruning.rs:6-29                                :func:`prune`
``networking``      networking.rs:5-120                            :func:`networking`
``toposort``        toposort.rs:4-39                               :func:`toposort`
``wellformed``      well_formed.rs:13-123                          :func:`well_formed`
``print``           print.rs:15-88 (DOT graph)                     :func:`print_graph`
``dump``            mod.rs:59-62 (textual dump)                    :func:`dump`
==================  =============================================  ===================

``compile(comp, passes=None, arg_specs=None)`` runs the default pipeline
(typing, deprecatedShape, lowering, prune, networking, toposort) or the named passes.
"""
from __future__ import annotations

import sys
from typing import Callable
from typing import Dict
from typing import List
from typing import Optional

from moose_amd import errors
from moose_amd.ir import types as T
from moose_amd.ir.computation import Computation
from moose_amd.ir.computation import HostPlacement
from moose_amd.ir.computation import Operation
from moose_amd.ir.computation import Signature
from moose_amd.ir.computation import rendezvous_key_from_counter

DEFAULT_PASSES = ["typing", "deprecatedShape", "lowering", "prune", "networking", "toposort"]


class CompilationError(errors.Compilation):
    pass


# ---------------------------------------------------------------------------
def typing_pass(comp: Computation, **_) -> Computation:
    """Fill Unknown argument types from the producers' return types (one hop)."""
    by_name = comp.by_name()
    out = []
    for op in comp.operations:
        args = list(op.sig.args)
        if op.sig.variadic:
            if args and args[0].name == "Unknown" and op.inputs:
                args = [by_name[op.inputs[0]].sig.ret]
        else:
            if len(args) < len(op.inputs):
                args = args + [T.Ty("Unknown")] * (len(op.inputs) - len(args))
            for i, inp in enumerate(op.inputs):
                src = by_name.get(inp)
                if src is None:
                    raise CompilationError(f"Could not find type of input {inp}")
                if args[i].name == "Unknown" or (
                        args[i].name == "Tensor" and args[i].inner is not None
                        and args[i].inner.kind == "Unknown"):
                    args[i] = src.sig.ret
        out.append(Operation(op.name, op.kind, list(op.inputs), op.placement,
                             Signature(tuple(args), op.sig.ret, op.sig.variadic), dict(op.attrs)))
    return Computation(out)


def deprecated_shape(comp: Computation, **_) -> Computation:
    """HostShape on logical-level Shape/Ones/Slice -> Shape<Host>."""
    host_shape, logical_shape = T.Ty("HostShape"), T.Ty("Shape", "Host")
    out = []
    for op in comp.operations:
        sig = op.sig
        if op.kind == "Shape" and sig.args and sig.args[0].name == "Tensor" and sig.ret == host_shape:
            sig = Signature(sig.args, logical_shape)
        elif op.kind == "Ones" and sig.ret.name == "Tensor" and sig.args and sig.args[0] == host_shape:
            sig = Signature((logical_shape,), sig.ret)
        elif op.kind == "Slice" and sig.args and sig.args[0] == host_shape and sig.ret == host_shape:
            sig = Signature((logical_shape,), logical_shape)
        out.append(Operation(op.name, op.kind, list(op.inputs), op.placement, sig, dict(op.attrs)))
    return Computation(out)


def lowering(comp: Computation, arg_specs=None, fixedpoint_ring: int = 128, **_) -> Computation:
    """Logical -> host-only graph by running the protocols on a SymbolicSession."""
    from moose_amd.compiler.symbolic import SymbolicSession
    from moose_amd.runtime.interpreter import Interpreter

    if is_lowered(comp):
        return comp
    sess = SymbolicSession(fixedpoint_ring)
    interp = Interpreter(sess, {}, fixedpoint_ring)
    interp.arg_specs = _norm_specs(arg_specs)
    interp.run(comp, {})
    return sess.computation()


def is_lowered(comp: Computation) -> bool:
    return all(isinstance(op.placement, HostPlacement) for op in comp.operations) and not any(
        op.sig.ret.name in ("Tensor", "Shape") or
        any(a.name in ("Tensor", "Shape") for a in op.sig.args) for op in comp.operations)


def _norm_specs(specs):
    out = {}
    for k, v in (specs or {}).items():
        if isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], (tuple, list)):
            out[k] = (tuple(v[0]), v[1])
        else:
            out[k] = (tuple(v), None)
    return out


def prune(comp: Computation, **_) -> Computation:
    """Operations that Outputs (and Saves) transitively depend on, following
    Send->Receive edges too (native graph core when available)."""
    from moose_amd.runtime import native_rt

    if native_rt.enabled():
        return native_rt.prune(comp)
    by_name = comp.by_name()
    roots = [op.name for op in comp.operations if op.kind in ("Output", "Save")]
    keep = set()
    stack = list(roots)
    while stack:
        n = stack.pop()
        if n in keep:
            continue
        keep.add(n)
        stack.extend(by_name[n].inputs)
    # keep Send/Receive pairs whose receiver survives
    return Computation([op for op in comp.operations if op.name in keep])


def networking(comp: Computation, **_) -> Computation:
    """Insert a Send/Receive pair for every (producer, consumer host) edge that crosses
    hosts; one pair per producer and destination host (reference networking.rs cache)."""
    by_name = comp.by_name()
    counter = 0
    cache: Dict[tuple, str] = {}
    extra: List[Operation] = []
    out = []
    for op in comp.operations:
        host = op.placement.owner if isinstance(op.placement, HostPlacement) else None
        if host is None:
            raise CompilationError("networking pass requires a lowered (host-only) computation")
        new_inputs = []
        for inp in op.inputs:
            src = by_name[inp]
            src_host = src.placement.owner
            if src_host == host:
                new_inputs.append(inp)
                continue
            key = (inp, host)
            if key not in cache:
                rdv = rendezvous_key_from_counter(counter)
                counter += 1
                send = Operation(f"send_{counter - 1}", "Send", [inp], HostPlacement(src_host),
                                 Signature((src.sig.ret,), T.Ty("HostUnit")),
                                 {"rendezvous_key": rdv, "receiver": host})
                recv = Operation(f"receive_{counter - 1}", "Receive", [], HostPlacement(host),
                                 Signature((), src.sig.ret),
                                 {"rendezvous_key": rdv, "sender": src_host})
                extra.extend([send, recv])
                cache[key] = recv.name
            new_inputs.append(cache[key])
        out.append(Operation(op.name, op.kind, new_inputs, op.placement, op.sig, dict(op.attrs)))
    return Computation(out + extra)


def toposort(comp: Computation, **_) -> Computation:
    return comp.toposorted()


_NO_KERNEL_CHECK = {"Load", "Save", "Send", "Receive"}  # as well_formed.rs:31
# host operations the graph executor runs itself (runtime/graph_executor.py _exec)
_HOST_EXECUTOR_OPS = {"Constant", "Input", "Output", "PrfKeyGen", "RingMulCross",
                      "BitAndCross", "RingDotCross"}
_PLAIN_TYPES = {"Unknown", "HostUnit", "HostString", "HostSeed", "HostPrfKey", "HostShape",
                "Shape", "Tensor", "Bit", "Float32", "Float64", "Ring64", "Ring128", "Fixed"}


def _types_compatible(expected: T.Ty, found: T.Ty) -> bool:
    if expected == found or "Unknown" in (expected.name, found.name):
        return True
    if expected.name == found.name == "Tensor":
        return T.UNKNOWN_DTYPE in (expected.inner, found.inner) or expected.inner is None \
            or found.inner is None
    shapes = {("HostShape", None), ("Shape", "Host"), ("Shape", "Unknown"), ("Shape", None)}
    return (expected.name, expected.inner) in shapes and (found.name, found.inner) in shapes


def _kernel_error(op) -> Optional[str]:
    """Why no kernel of this executor runs ``op`` at its placement and signature, or None:
    the static counterpart of the interpreter's routing (declarative table for ring-level
    replicated / additive ops, replicated dialect protocols, logical op_* handlers, host
    primitives) -- the role of DispatchKernel::compile in well_formed.rs:28-116."""
    from moose_amd.ir.computation import AdditivePlacement
    from moose_amd.ir.computation import ReplicatedPlacement
    from moose_amd.runtime import dispatch
    from moose_amd.runtime import interpreter as I
    from moose_amd.runtime.prims import PRIMS

    if op.kind in _NO_KERNEL_CHECK or op.sig is None:
        return None
    plc = op.placement
    args = [t.name for t in op.sig.args]
    if op.sig.variadic and args:
        args = args[:1] * max(1, len(op.inputs))
    concrete = any(a not in _PLAIN_TYPES for a in args) or op.sig.ret.name not in _PLAIN_TYPES
    logical = getattr(I.Interpreter, f"op_{op.kind}", None) is not None
    if isinstance(plc, AdditivePlacement):
        if dispatch.lookup(op.kind, "adt", args) is not None:
            return None
        return f"no additive kernel for {op.kind} on ({', '.join(args)})"
    if isinstance(plc, ReplicatedPlacement):
        if dispatch.lookup(op.kind, "rep", args) is not None or op.kind in I._REP_DIALECT:
            return None
        if logical and not any(a.startswith(("Additive", "Host")) for a in args):
            return None
        return f"no replicated kernel for {op.kind} on ({', '.join(args)})"
    if isinstance(plc, HostPlacement):
        if op.kind == "Reveal" and dispatch.lookup("Reveal", "host", args) is not None:
            return None
        if logical or op.kind in PRIMS or op.kind in _HOST_EXECUTOR_OPS:
            return None
        return f"no host kernel for {op.kind}"
    # mirrored placements run the logical handlers
    if logical or (not concrete and op.kind in PRIMS):
        return None
    return f"no kernel for {op.kind} on {type(plc).__name__}"


def well_formed(comp: Computation, **_) -> Computation:
    """Topological order, every operator known, every input defined earlier, argument
    counts and producer types consistent with each signature, and a kernel for every
    (operator, placement, signature) instantiation (reference well_formed.rs:13-123)."""
    from moose_amd.ir.operators import ALL_OPERATORS
    from moose_amd.runtime import native_rt

    if native_rt.enabled():
        try:
            bad = native_rt.graph_of(comp).first_out_of_order()
        except (native_rt.mod().NativeGraphError, KeyError) as e:
            raise CompilationError(str(e)) from None
        if bad >= 0:
            op = comp.operations[bad]
            raise CompilationError(f"{op.name}: an input is not defined before use")

    seen = {}
    sends = {bytes(op.attrs["rendezvous_key"]) for op in comp.operations if op.kind == "Send"}
    for op in comp.operations:
        if op.kind not in ALL_OPERATORS:
            raise CompilationError(f"{op.name}: unknown operator {op.kind}")
        for i in op.inputs:
            if i not in seen:
                raise CompilationError(f"{op.name}: input {i} is not defined before use")
        if op.kind == "Receive" and bytes(op.attrs["rendezvous_key"]) not in sends:
            raise CompilationError(f"{op.name}: no Send for its rendezvous key")
        if op.name in seen:
            raise CompilationError(f"duplicate operation name {op.name}")
        sig = op.sig
        if sig is not None and sig.args:
            if not sig.variadic and len(sig.args) != len(op.inputs):
                raise CompilationError(f"{op.name}: {op.kind} takes {len(sig.args)} "
                                       f"argument(s), {len(op.inputs)} given")
            for k, i in enumerate(op.inputs):
                want = sig.args[0] if sig.variadic else sig.args[k]
                got = seen[i].sig.ret if seen[i].sig is not None else T.UNKNOWN
                if not _types_compatible(want, got):
                    raise CompilationError(
                        f"{op.name}: argument {k} ({i}): "
                        f"{errors.TypeMismatch(want.to_textual(), got.to_textual())}")
        why = _kernel_error(op)
        if why is not None:
            raise CompilationError(f"{op.name}: {why}")
        seen[op.name] = op
    return comp


_COLORS = ["#336699", "#ff0000", "#ff6600", "#92cd00", "#ffcc00", "#7f00ff", "#00994d"]


def to_dot(comp: Computation) -> str:
    roles = sorted({r for op in comp.operations for r in _owners(op.placement)})
    color = {r: _COLORS[i % len(_COLORS)] for i, r in enumerate(roles)}
    lines = ["digraph {"]
    for op in comp.operations:
        c = color[_owners(op.placement)[0]]
        lines.append(f'    "{op.name}" [label="{op.name} = {op.kind}\\n'
                     f'{op.placement.to_textual()}" color="{c}" shape=rectangle]')
    for op in comp.operations:
        for i in op.inputs:
            lines.append(f'    "{i}" -> "{op.name}"')
    lines.append("}")
    return "\n".join(lines)


def _owners(plc):
    return (plc.owner,) if isinstance(plc, HostPlacement) else tuple(plc.owners)


def print_graph(comp: Computation, out=None, **_) -> Computation:
    (out or sys.stdout).write(to_dot(comp) + "\n")
    return comp


def dump(comp: Computation, out=None, **_) -> Computation:
    (out or sys.stdout).write(comp.to_textual() + "\n")
    return comp


PASSES: Dict[str, Callable] = {
    "typing": typing_pass,
    "deprecatedShape": deprecated_shape,
    "lowering": lowering,
    "prune": prune,
    "networking": networking,
    "toposort": toposort,
    "wellformed": well_formed,
    "print": print_graph,
    "dump": dump,
}


_PLAN_CACHE: Dict[str, Computation] = {}
_PLAN_CACHE_MAX = 32


def _plan_key(comp, names, arg_specs, fixedpoint_ring):
    import hashlib

    spec = sorted((k, str(v)) for k, v in (arg_specs or {}).items())
    h = hashlib.blake2b(digest_size=16)
    for part in (comp.digest(), ",".join(names), repr(spec), str(fixedpoint_ring)):
        h.update(part.encode())
    return h.hexdigest()


def compile(comp: Computation, passes: Optional[List[str]] = None,  # noqa: A001
            arg_specs=None, fixedpoint_ring: int = 128, cache: bool = True) -> Computation:
    """Run the pass pipeline.  Lowered plans are deterministic (PRF nonces are counters,
    not random sync keys), so results are cached by (computation digest, passes, input
    shapes, ring) in memory and, with ``MOOSEX_PLAN_CACHE=<dir>``, on disk."""
    import os

    names = DEFAULT_PASSES if passes is None else list(passes)
    for name in names:
        if name not in PASSES:
            raise CompilationError(f"Unknown pass requested: {name}")
    side_effects = any(n in ("print", "dump") for n in names)
    key = _plan_key(comp, names, arg_specs, fixedpoint_ring) if cache and not side_effects else None
    if key is not None:
        hit = _PLAN_CACHE.get(key)
        if hit is not None:
            return hit
        disk = os.environ.get("MOOSEX_PLAN_CACHE")
        if disk and os.path.exists(os.path.join(disk, key + ".msgpack")):
            plan = Computation.from_disk(os.path.join(disk, key + ".msgpack"))
            _PLAN_CACHE[key] = plan
            return plan
    for name in names:
        comp = PASSES[name](comp, arg_specs=arg_specs, fixedpoint_ring=fixedpoint_ring)
    if key is not None:
        if len(_PLAN_CACHE) >= _PLAN_CACHE_MAX:
            _PLAN_CACHE.pop(next(iter(_PLAN_CACHE)))
        _PLAN_CACHE[key] = comp
        disk = os.environ.get("MOOSEX_PLAN_CACHE")
        if disk:
            os.makedirs(disk, exist_ok=True)
            comp.to_disk(os.path.join(disk, key + ".msgpack"))
    return comp
