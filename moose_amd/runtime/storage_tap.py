"""Storage-backed computations in replayed evaluations (hipGraph plans, per-party tapes).

The reference runs ``Load`` / ``Save`` as ordinary dataflow tasks of the session
(``/root/reference/moose/src/execution/asynchronous.rs:149-238, 456-466``; the storage
trait: ``/root/reference/moose/src/storage/mod.rs:10-33``): a worker fed from its storage --
the comet / rudolph deployments, the linear-regression example -- evaluates like any other.
A replay cannot call back into Python storage from inside a graph, so a
:class:`StorageTap` moves the storage accesses to the replay's edges, exactly as arguments
and outputs are handled:

* every host ``Load`` whose key is a constant or a string argument is a static device
  buffer, filled from the storage before the capture and refreshed from it before each
  replay (a copy, like an argument; a stored value whose shape or dtype changed gives
  another signature, so the runtime captures again);
* every host ``Save`` is recorded at capture as the value it stores; after each replay the
  value is read back and written to the storage (like an output).

Loaded strings and scalars are captured as constants and are part of the signature.  A
``Load`` of a key the same evaluation ``Save``s first would need the saved value inside the
graph: not capturable (the evaluation stays eager), as are share checkpoints on replicated
placements and loads whose key is computed.
"""
from __future__ import annotations

from typing import Dict
from typing import Optional

import numpy as np
import torch

from moose_amd import errors
from moose_amd.ir.computation import HostPlacement


class TapeUnsupported(errors.Unexpected):
    """The computation's storage accesses cannot be replayed (it is evaluated eagerly)."""


def _key_source(ops: Dict[str, object], name: str):
    """Where a Load / Save key comes from: ("const", text) for a string constant, ("arg",
    argument name) for a string argument (part of a plan's argument signature), None for a
    computed key."""
    op = ops.get(name)
    if op is None:
        return None
    if op.kind == "Constant":
        c = op.attrs.get("value")
        v = getattr(c, "value", c)
        return ("const", v) if isinstance(v, str) else None
    if op.kind == "Input":
        return ("arg", op.attrs.get("arg_name") or op.name)
    return None


def _resolve(src, arguments):
    if src is None:
        return None
    if src[0] == "const":
        return src[1]
    v = (arguments or {}).get(src[1])
    return v if isinstance(v, str) else None


_PLANS: Dict[int, tuple] = {}


def _structure(comp):
    """(loads, saves) with key sources, cached per computation object; an Exception value
    when a replay cannot serve them."""
    hit = _PLANS.get(id(comp))
    if hit is not None and hit[0] is comp:
        return hit[1]
    ops = {op.name: op for op in comp.operations}
    loads, saves, res = [], [], None
    for op in comp.operations:
        if op.kind not in ("Load", "Save"):
            continue
        if not isinstance(op.placement, HostPlacement):
            res = TapeUnsupported(f"{op.kind} {op.name} on {op.placement}: share checkpoints "
                                  "are evaluated eagerly")
            break
        key = _key_source(ops, op.inputs[0]) if op.inputs else None
        if key is None:
            res = TapeUnsupported(f"{op.kind} {op.name}: its key is computed")
            break
        host = op.placement.owner
        if op.kind == "Load":
            query = _key_source(ops, op.inputs[1]) if len(op.inputs) > 1 else None
            loads.append((op.name, host, key, query))
        else:
            saves.append((op.name, host, key))
    if res is None:
        res = (loads, saves)
    if len(_PLANS) > 256:
        _PLANS.clear()
    _PLANS[id(comp)] = (comp, res)
    return res


def storage_ops(comp, arguments=None):
    """``(loads, saves)`` of ``comp`` with its keys resolved against ``arguments``:
    [(op name, host, key, query)] and [(op name, host, key)] for its host-placement Load /
    Save ops.  Raises TapeUnsupported for accesses a replay cannot serve (share
    checkpoints, computed keys, a key the evaluation both saves and loads)."""
    st = _structure(comp)
    if isinstance(st, Exception):
        raise st
    loads, saves = [], []
    for name, host, src, qsrc in st[0]:
        key = _resolve(src, arguments)
        if key is None:
            raise TapeUnsupported(f"Load {name}: its key argument is not a string")
        loads.append((name, host, key, _resolve(qsrc, arguments) or ""))
    for name, host, src in st[1]:
        key = _resolve(src, arguments)
        if key is None:
            raise TapeUnsupported(f"Save {name}: its key argument is not a string")
        saves.append((name, host, key))
    saved = {(h, k) for _, h, k in saves}
    for name, host, key, _q in loads:
        if (host, key) in saved:
            raise TapeUnsupported(f"Load {name}: key {key!r} is also saved by the evaluation")
    return loads, saves


def capturable(comp, arguments=None) -> bool:
    """Can a replay serve ``comp``'s storage accesses?  Without ``arguments`` only the
    structure is checked (keys from arguments are resolved per evaluation)."""
    try:
        if arguments is None:
            st = _structure(comp)
            if isinstance(st, Exception):
                raise st
        else:
            storage_ops(comp, arguments)
    except TapeUnsupported:
        return False
    return True


def fetch(storage, host: str, key: str, query: str = ""):
    """The value a Load of ``key`` on ``host`` reads (interpreter.op_Load's rule)."""
    store = storage.get(host, {}) if storage is not None else {}
    if key in store:
        return store[key]
    from moose_amd.utils import storage as st

    value = st.load_from_path(key, query) if st.looks_like_path(key) else None
    if value is None:
        raise errors.MooseRuntimeError(f"key {key!r} not found in storage of {host}")
    return value


def _is_array(v) -> bool:
    return isinstance(v, (np.ndarray, np.generic)) or (
        isinstance(v, (list, tuple)) and bool(v) and not isinstance(v[0], (str, bytes)))


def _sig_of(v):
    if isinstance(v, torch.Tensor):
        return ("tensor", tuple(v.shape), str(v.dtype))
    if _is_array(v):
        a = np.asarray(v)
        return ("array", a.shape, a.dtype.str)
    return ("value", repr(v))


def signature(comp, storage, hosts: Optional[set] = None, arguments=None):
    """Hashable description of what ``comp``'s Loads read from ``storage`` (restricted to
    ``hosts`` when given): () when it loads nothing.  A replay is specialised on it."""
    try:
        loads, _ = storage_ops(comp, arguments)
    except TapeUnsupported:
        return ("eager",)
    sig = []
    for _name, host, key, query in loads:
        if hosts is not None and host not in hosts:
            continue
        try:
            sig.append((host, key, _sig_of(fetch(storage, host, key, query))))
        except errors.MooseRuntimeError:
            sig.append((host, key, None))
    return tuple(sig)


class StorageTap:
    """The storage accesses of one captured evaluation (module docstring).  ``hosts``: the
    placements this process evaluates (one-process-per-party tapes); None = all."""

    def __init__(self, comp, storage, device, hosts: Optional[set] = None, arguments=None):
        from moose_amd.runtime.interpreter import dtype_of_numpy
        from moose_amd.runtime.interpreter import numpy_to_torch

        loads, saves = storage_ops(comp, arguments)
        self.device = torch.device(device)
        mine = (lambda h: True) if hosts is None else (lambda h: h in hosts)  # noqa: E731
        self.loads = [(h, k, q) for _n, h, k, q in loads if mine(h)]
        self.save_keys = [(h, k) for _n, h, k in saves if mine(h)]
        self.static = {}  # (host, key) -> device tensor or captured python value
        for host, key, query in self.loads:
            v = fetch(storage, host, key, query)
            if isinstance(v, torch.Tensor):
                t = v.detach().to(self.device).clone()
                t._moose_dtype = getattr(v, "_moose_dtype", None)
                self.static[(host, key)] = t
            elif _is_array(v):
                a = np.asarray(v)
                t = numpy_to_torch(a, self.device)
                t._moose_dtype = dtype_of_numpy(a)
                self.static[(host, key)] = t
            else:
                self.static[(host, key)] = v
        self.saves = []  # (host, key, interpreter, value) recorded during the capture

    # -- during the capture (interpreter.op_Load / op_Save) ---------------------------------
    def load(self, host: str, key: str):
        try:
            return self.static[(host, key)]
        except KeyError:
            raise TapeUnsupported(f"Load of {key!r} on {host} was not staged") from None

    def record_save(self, host: str, key: str, interp, lv):
        self.saves.append((host, key, interp, lv))

    # -- around each replay -----------------------------------------------------------------
    def refresh(self, storage):
        """Copy the current stored values into the static buffers (the current stream).
        A value of another shape, dtype or (for captured scalars) value raises
        TapeUnsupported: the caller's signature check should have re-captured."""
        for host, key, query in self.loads:
            v = fetch(storage, host, key, query)
            t = self.static[(host, key)]
            if not isinstance(t, torch.Tensor):
                if repr(v) != repr(t):
                    raise TapeUnsupported(f"stored {key!r} changed: captured as a constant")
                continue
            if isinstance(v, torch.Tensor):
                src = v.detach()
            else:
                a = np.asarray(v)
                a = a.view(np.int64) if a.dtype == np.uint64 else a
                src = torch.from_numpy(np.ascontiguousarray(a))
            if tuple(src.shape) != tuple(t.shape):
                raise TapeUnsupported(f"stored {key!r} changed shape")
            if src.dtype != t.dtype:
                if src.is_floating_point() != t.is_floating_point():
                    raise TapeUnsupported(f"stored {key!r} changed dtype")
                src = src.to(t.dtype)
            t.copy_(src)

    def write_saves(self, storage):
        """Read back every value the evaluation saves and store it (after the replay)."""
        for host, key, interp, lv in self.saves:
            if interp.sess.materialized(lv.v):
                storage.setdefault(host, {})[key] = interp.to_numpy(lv)


def storage_fed(comp, names):
    """``comp`` with its arguments ``names`` read from storage instead: each such Input op
    becomes a Load of the key <argument name> on the same placement (the deployment where a
    worker's data sits in its storage, as the reference's comet / rudolph workers).  Used by
    the bench's storage-fed LR record and the tests."""
    from moose_amd.ir.computation import Computation
    from moose_amd.ir.computation import Constant
    from moose_amd.ir.computation import Operation
    from moose_amd.ir.computation import Signature
    from moose_amd.ir.types import Ty

    text = Ty("HostString")
    ops = []
    for op in comp.operations:
        arg = op.attrs.get("arg_name") or op.name if op.kind == "Input" else None
        if arg is None or arg not in names or not isinstance(op.placement, HostPlacement):
            ops.append(op)
            continue
        k, q = f"{op.name}__key", f"{op.name}__query"
        ops.append(Operation(k, "Constant", [], op.placement, Signature((), text),
                             {"value": Constant("HostString", arg)}))
        ops.append(Operation(q, "Constant", [], op.placement, Signature((), text),
                             {"value": Constant("HostString", "")}))
        ops.append(Operation(op.name, "Load", [k, q], op.placement,
                             Signature((text, text), op.sig.ret), {}))
    return Computation(ops)
