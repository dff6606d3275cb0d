"""Logical interpreter: evaluate a (logical-level) native-IR computation on a session.

Each logical operator is dispatched on its placement kind, exactly like the
reference's logical kernels (``moose/src/logical/ops.rs``: ``logical_host_kernel`` /
``logical_rep_kernel``) and fixed-point kernels (``moose/src/fixedpoint/ops.rs``):
inputs are implicitly converted to the op's placement (share host values onto a
replicated placement, reveal replicated values to a host, mirror/demirror), fixed-point
products are followed by a truncation, and comparisons return boolean sharings.

Unlike the reference, the replicated path is *not* first lowered to thousands of host
ops: every replicated op runs its fused protocol directly on the session (one stacked
kernel per local step on a single MI355X, RCCL send/recv between MI355Xs), which is the
fast path used by ``LocalMooseRuntime`` and the benchmarks.  Lowering to a host graph
is still available (``moose_amd.compiler``) and runs the same protocol code on a
symbolic session.
"""
from __future__ import annotations

import functools
import math
import os
import threading
from typing import Dict

import numpy as np
import torch

from moose_amd import errors
from moose_amd.ir import types as T
from moose_amd.ir.computation import Computation
from moose_amd.ir.computation import Constant
from moose_amd.ir.computation import HostPlacement
from moose_amd.ir.computation import Mirrored3Placement
from moose_amd.ir.computation import Operation
from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ops import ring as R
from moose_amd.protocols import fixedpoint as fxp
from moose_amd.protocols import replicated as rep
from moose_amd.protocols.fixedpoint import RepFixed
from moose_amd.runtime import lanes as _lanes
from moose_amd.runtime import shares
from moose_amd.runtime.session import HV
from moose_amd.runtime.session import nonce_scope
from moose_amd.runtime.values import LV
from moose_amd.runtime.values import MV
from moose_amd.utils.telemetry import span

_FLOAT = {"Float32": torch.float32, "Float64": torch.float64}
# small numeric tensor constants of computations, uploaded once per (value, device)
_CONST_LV = {}
_CONST_LOCK = threading.Lock()
# multi-round elementwise ops merged across independent chains (Interpreter._merge_unary)
_MERGE_KINDS = {"Sigmoid", "Exp", "Log", "Log2", "Sqrt", "Relu", "Abs"}
# multi-round operations that independent ops of OTHER kinds may run beside in lockstep
# (parallel/lockstep.py): their message rounds are merged
_LOCKSTEP_KINDS = _MERGE_KINDS | {"Div", "Less", "Greater", "Softmax", "Argmax", "Maximum",
                                  "Dot", "Mul", "Pow2", "Msb", "Equal", "Mux", "Sign",
                                  "TruncPr", "BitDecompose", "Mean", "Sum", "AddN"}
LOCKSTEP = os.environ.get("MOOSEX_LOCKSTEP", "1") != "0"
_MERGE_FNS = {"Sigmoid": fxp.sigmoid, "Exp": fxp.exp, "Log": fxp.log, "Log2": fxp.log2,
              "Sqrt": fxp.sqrt, "Relu": fxp.relu, "Abs": fxp.abs_}
MERGE_ROUNDS = os.environ.get("MOOSEX_MERGE_ROUNDS", "1") != "0"
# per-operation nonce scopes (runtime/session.py nonce_scope; MOOSEX_NONCE_SCOPES=0: one
# session-wide counter, the round-5 numbering)
NONCE_SCOPES = os.environ.get("MOOSEX_NONCE_SCOPES", "1") != "0"
# operand + output elements of one batched Dot call (Interpreter._batch_dots)
BATCH_DOT_ELEMS = int(os.environ.get("MOOSEX_BATCH_DOT_ELEMS", str(1 << 25)))
# per-party sessions broadcast a one-element secret operand of add / sub / mul inside the
# kernels instead of materialising it (MOOSEX_BCAST_IN_KERNEL=0: materialised)
BCAST_IN_KERNEL = os.environ.get("MOOSEX_BCAST_IN_KERNEL", "1") != "0"


def _by_depth(ops):
    """A topological order by depth (longest path from a source), stable within a depth:
    operations that do not depend on each other and sit at the same depth become adjacent,
    so the merge of independent chains finds their inputs computed.  A deterministic
    function of the computation: every process of an SPMD job runs the same order."""
    depth = {}
    for op in ops:  # ``ops`` is already topologically sorted
        depth[op.name] = 1 + max((depth.get(n, 0) for n in op.inputs), default=0)
    order = sorted(range(len(ops)), key=lambda i: (depth[ops[i].name], i))
    return [ops[i] for i in order]


# replicated dialect operators handled by Interpreter._rep_dialect (reference
# replicated/{convert,arith,bits,compare}.rs; Share/TruncPr are special-cased there)
_REP_DIALECT = {
    "Share": None, "TruncPr": None,
    "Msb": rep.msb, "BitDecompose": rep.bit_decompose, "EqualZero": rep.equal_zero,
    "Xor": rep.xor, "And": rep.and_, "Shl": rep.shl, "BitExtract": rep.bit_extract,
    "RingInject": rep.b2a, "Equal": rep.equal, "Index": rep.bit_extract,
}


# argument types of logical-level operations: the dispatch table only holds ring-level rows
_LOGICAL_TY = frozenset({"Tensor", "Shape", "Unknown", "HostShape", "HostUnit", "HostString",
                         "HostSeed", "HostPrfKey", "Float32", "Float64"})


class MooseRuntimeError(errors.KernelError):
    pass


def _owners(plc):
    return (plc.owner,) if isinstance(plc, HostPlacement) else tuple(plc.owners)


def torch_dtype_of(dtype: T.TensorDType):
    k = dtype.kind
    if k in _FLOAT:
        return _FLOAT[k]
    if k == "Bool":
        return torch.bool
    if k == "Uint64":
        return torch.int64
    raise MooseRuntimeError(f"no plaintext torch dtype for {dtype}")


def dtype_of_numpy(a: np.ndarray) -> T.TensorDType:
    m = {
        np.dtype("float64"): T.FLOAT64,
        np.dtype("float32"): T.FLOAT32,
        np.dtype("bool"): T.BOOL,
        np.dtype("uint64"): T.UINT64,
    }
    if a.dtype in m:
        return m[a.dtype]
    if np.issubdtype(a.dtype, np.integer):
        return T.TensorDType("Uint64") if a.dtype.kind == "u" else T.TensorDType("Int64")
    raise MooseRuntimeError(f"unsupported numpy dtype {a.dtype}")


def numpy_to_torch(a, device):
    a = np.asarray(a)
    if a.dtype == np.uint64:
        return R.to_device(torch.from_numpy(a.view(np.int64).copy()), device)
    if a.dtype == np.uint32:
        a = a.astype(np.int64)
    elif a.dtype == np.uint16:
        a = a.astype(np.int32)
    if a.dtype == object:
        raise MooseRuntimeError("object arrays are not tensors")
    return R.to_device(torch.from_numpy(np.ascontiguousarray(a)), device)


class Interpreter:
    def __init__(self, sess, storage=None, fixedpoint_ring: int = None, lanes: int = None):
        self.sess = sess
        self.storage = storage if storage is not None else {}
        self.env: Dict[str, LV] = {}
        self.fixed_ring = fixedpoint_ring  # override Fixed128 -> Fixed64 if 64
        self.outputs = {}
        self.on_op = None
        # replayed evaluations: Load / Save served by a runtime.storage_tap.StorageTap
        self.storage_tap = None
        # independent operations on separate HIP streams (runtime/lanes.py)
        self.lanes = None
        dev = getattr(sess, "device", None)
        n = lanes if lanes is not None else _lanes.default_lanes()
        if n > 1 and dev is not None and dev.type == "cuda" and getattr(sess, "me", None) is None:
            self.lanes = _lanes.LaneRunner(dev, n)

    # ------------------------------------------------------------------------
    # driver
    # ------------------------------------------------------------------------
    def run(self, comp: Computation, arguments: dict) -> dict:
        self.arguments = arguments or {}
        self._at_memo = {}
        comp = comp.toposorted()
        # every non-host operation draws its PRF nonces from a scope of its own, numbered by
        # its place among them in the toposorted program (the same on every party and in
        # every layout; host operations -- which draw none -- do not shift the numbering)
        self._scope = {op.name: i + 1 for i, op in enumerate(
            o for o in comp.operations if not isinstance(o.placement, HostPlacement))}
        me = getattr(self.sess, "me", None)  # set for one-process-per-party sessions
        batch = getattr(self.sess, "batch_dots", False) and os.environ.get(
            "MOOSEX_BATCH_DOTS", "1") != "0"
        ops = comp.operations
        if (MERGE_ROUNDS and getattr(self.sess, "merge_rounds", False)
                and not any(op.kind in ("Save", "Load") for op in ops)):
            ops = _by_depth(ops)  # independent ops of one depth adjacent (_merge_unary)
        lanes = self.lanes
        begin = getattr(self.sess, "begin_evaluation", None)
        if begin is not None:
            begin(comp, self.arguments)
        ok = False
        if lanes is not None:
            lanes.start(ops)
        try:
            for idx, op in enumerate(ops):
                if op.name in self.env:  # computed ahead as part of a batch
                    continue
                if self.on_op is not None:  # e.g. graph capture segmentation (graphs.py)
                    self.on_op()
                if lanes is not None:
                    lanes.enter(op, self.env)
                    before = len(self.env)
                try:
                    self._run_op(op, ops, idx, batch, me)
                finally:
                    if lanes is not None:
                        lanes.leave([n for n in list(self.env)[before:]])
            ok = True
        finally:
            if lanes is not None:
                lanes.finish()
            release = getattr(self.sess, "end_evaluation", None)
            if release is not None:
                release(ok)
        return self.outputs

    def _run_op(self, op, ops, idx, batch, me):
        with nonce_scope(self._scope.get(op.name) if NONCE_SCOPES else None):
            self._run_op_scoped(op, ops, idx, batch, me)

    def _run_op_scoped(self, op, ops, idx, batch, me):
        table = self._table_handler(op)
        if (table is None and batch and op.kind == "Dot"
                and self._batch_dots(op, ops[idx + 1:])):
            return
        if (table is None and LOCKSTEP and op.kind in _LOCKSTEP_KINDS
                and getattr(self.sess, "merge_rounds", False) and self.lanes is None
                and self._lockstep(op, ops[idx + 1:], me)):
            return
        if (table is None and op.kind in _MERGE_KINDS and MERGE_ROUNDS
                and getattr(self.sess, "merge_rounds", False)
                and self._merge_unary(op, ops[idx + 1:])):
            return
        handler = table or getattr(self, f"op_{op.kind}", None) or self._dialect_handler(op)
        if handler is None:
            raise MooseRuntimeError(f"operator {op.kind} is not supported by the interpreter")
        ins = [self.env[n] for n in op.inputs]
        with span(f"op.{op.kind}", op=op.name):
            try:
                if me is not None and me not in _owners(op.placement):
                    self.env[op.name] = self._foreign_op(op, ins, me)
                else:
                    self.env[op.name] = handler(op, ins)
            except MooseRuntimeError:
                raise
            except Exception as e:  # annotate with the failing op
                raise MooseRuntimeError(f"{op.name} = {op.kind} failed: {e}") from e

    def _batch_dots(self, op, later, limit: int = 256) -> bool:
        """Independent-op batching (the reference runs independent operations as
        concurrent tasks, execution/asynchronous.rs:456-530): a secret x secret
        fixed-point Dot on a replicated placement is executed together with every later
        Dot whose operands are already computed (so none depends on another) and have the
        same placement, dtype and shapes -- one batched GEMM / reshare / TruncPr for all
        (fixedpoint.dot_many).  Returns False when there is nothing to batch."""
        def key(o):
            if not isinstance(o.placement, ReplicatedPlacement):
                return None
            if any(n not in self.env for n in o.inputs):
                return None
            x, y = (self._at_memo_put(o, self.env[n]) for n in o.inputs)
            if x.kind != "tensor" or y.kind != "tensor" or x.dtype is None:
                return None
            if not x.dtype.is_fixed or x.dtype != y.dtype or x.is_host or x.is_mir or y.is_mir:
                return None
            if self._public(x) is not None or self._public(y) is not None:
                return None
            try:
                sx, sy = fxp.shape_of(self.sess, x.v), fxp.shape_of(self.sess, y.v)
            except Exception:  # noqa: BLE001 - symbolic/unknown shapes: no batching
                return None
            if len(sx) != 2 or len(sy) != 2:
                return None
            return (o.placement, x.dtype, tuple(sx), tuple(sy)), x, y

        k0 = key(op)
        if k0 is None:
            return False
        group = [(op, k0[1], k0[2])]
        # one batched product stays within a bounded operand + output size (the batched GEMM
        # and its workspace grow with it: 100 products of 1000 x 1000 in one call asked for
        # tens of GiB); the rest are batched by the next Dot's call
        (_, _, sx, sy) = k0[0]
        per = sx[0] * sx[1] + sy[0] * sy[1] + sx[0] * sy[1]
        limit = max(1, min(limit, BATCH_DOT_ELEMS // max(1, per)))
        for o in later:
            if len(group) >= limit:
                break
            if o.kind != "Dot" or o.name in self.env or any(n not in self.env for n in o.inputs):
                continue
            if self.lanes is not None and not self.lanes.ordered_here(o.inputs):
                continue  # an operand from another lane this lane has not waited on
            if self._table_handler(o) is not None:
                continue
            k = key(o)
            if k is not None and k[0] == k0[0]:
                group.append((o, k[1], k[2]))
        if len(group) == 1:
            return False
        dtype = k0[1].dtype
        with span("op.Dot.batched", n=len(group)):
            outs = fxp.dot_many(self.sess, [(x.v, y.v) for _, x, y in group],
                                dtype.fractional_precision)
        for (o, x, _), r in zip(group, outs):
            if self.on_op is not None and self.lanes is None:
                self.on_op()
            self.env[o.name] = LV(x.plc, "tensor", dtype, r)
        return True

    def _lockstep(self, op, later, me, limit: int = 8) -> bool:
        """Intra-evaluation overlap of DIFFERENT kinds (parallel/lockstep.py): a multi-round
        replicated op runs as a coroutine beside the later ops of the lockstep kinds on the
        same placement whose inputs are already computed (independent of it and of each
        other); their message rounds go out merged, so the group costs the rounds of its
        longest member.  Same-kind elementwise ops inside the group still run as ONE merged
        protocol (a unit, as _merge_unary forms it).  Every unit's inputs are converted
        (e.g. host inputs shared) before the coroutines start, in program order and each
        under the nonce scope its one-by-one run uses, so the shares are bitwise those of
        running the units one by one.  MOOSEX_LOCKSTEP=0 disables it."""
        from moose_amd.parallel.lockstep import Lockstep

        plc = op.placement
        if not isinstance(plc, ReplicatedPlacement):
            return False
        # a process outside the placement forms the same units and converts the same inputs
        # (it takes part in sharing its own), then runs the units one by one
        member = me is None or me in _owners(plc)

        def ready(o):
            return (o.kind in _LOCKSTEP_KINDS and o.placement == plc and o.name not in self.env
                    and all(n in self.env for n in o.inputs) and self._table_handler(o) is None)

        if not ready(op):
            return False
        cands = [op]
        for o in later:
            if len(cands) >= limit:
                break
            if ready(o):
                cands.append(o)
        if len(cands) == 1:
            return False

        def mkey(o):  # _merge_unary's grouping, from the program's structure
            if not (MERGE_ROUNDS and o.kind in _MERGE_KINDS and len(o.inputs) == 1):
                return None
            x = self.env[o.inputs[0]]
            if x.kind != "tensor" or x.dtype is None or not x.dtype.is_fixed or x.is_mir:
                return None
            return (o.kind, x.dtype, repr(sorted(o.attrs.items())))

        units, used = [], set()
        for o in cands:
            if o.name in used:
                continue
            k = mkey(o)
            members = [o] + ([c for c in cands if c.name not in used and c is not o
                              and mkey(c) == k] if k is not None else [])
            used.update(m.name for m in members)
            units.append(members)
        if len(units) == 1:
            return False  # one same-kind group: _merge_unary's
        # a lazy replicated input (a product whose last rounds run when first read) that
        # several units read is settled first, under the scope of the first of them
        seen = {}
        for u in units:
            for o in u:
                for n in o.inputs:
                    if u[0].name not in seen.setdefault(n, []):
                        seen[n].append(u[0].name)
        for n, users in seen.items():
            t = getattr(self.env[n].v, "t", self.env[n].v)
            if len(users) > 1 and rep.lazy(t):
                with nonce_scope(self._scope.get(users[0])):
                    rep.settle(t)

        # inputs converted in program order, as the units' one-by-one runs would: a merged
        # unit through the batching memo (_merge_unary's probe: later units may reuse it), a
        # single op as its handler's ``at`` (consuming a memo entry), kept for that handler
        pre = self.__dict__.setdefault("_lockstep_pre", {})
        for u in units:
            with nonce_scope(self._scope.get(u[0].name)):
                for o in u:
                    for n in o.inputs:
                        lv = self.env[n]
                        if len(u) > 1:
                            self._at_memo_put(o, lv)
                            continue
                        conv = self.at(o, lv)
                        if conv is not lv:
                            pre[(o.name, id(lv))] = (lv, conv)

        def evaluate(o):
            handler = getattr(self, f"op_{o.kind}", None) or self._dialect_handler(o)
            if handler is None:
                raise MooseRuntimeError(f"operator {o.kind} is not supported by the interpreter")
            ins = [self.env[n] for n in o.inputs]
            with span(f"op.{o.kind}", op=o.name):
                try:
                    if not member:
                        return self._foreign_op(o, ins, me)
                    return handler(o, ins)
                except MooseRuntimeError:
                    raise
                except Exception as e:  # annotate with the failing op
                    raise MooseRuntimeError(f"{o.name} = {o.kind} failed: {e}") from e

        def run_unit(u):
            if len(u) == 1:
                return [(u[0], evaluate(u[0]))]
            group = [(o, self._at_memo_put(o, self.env[o.inputs[0]])) for o in u]
            return self._merge_compute(u[0].kind, group)

        try:
            with span("op.lockstep", n=len(units)):
                if member:
                    outs = Lockstep(self.sess).run(
                        [functools.partial(run_unit, u) for u in units],
                        [self._scope.get(u[0].name) for u in units])
                else:
                    outs = []
                    for u in units:
                        with nonce_scope(self._scope.get(u[0].name)):
                            outs.append(run_unit(u))
        finally:
            pre.clear()
        for res in outs:
            for o, lv in res:
                self.env[o.name] = lv
        return True

    def _merge_unary(self, op, later, limit: int = 16) -> bool:
        """Intra-evaluation overlap for one-party-per-process / per-thread sessions (the
        reference's async session overlaps independent operations,
        execution/asynchronous.rs:456-530): a multi-round elementwise fixed-point op
        (sigmoid, exp, log, sqrt, relu, ...) runs TOGETHER with every later op of the same
        kind, placement, dtype and attributes whose input is already computed -- the inputs
        flattened and concatenated, one protocol run, the result split back -- so k
        independent chains cost the rounds (message latencies) of one instead of k.  The
        grouping uses only the computation's structure, so every process of an SPMD job
        forms the same groups.  Values: each element's protocol run is the same
        computation; only the PRF streams and TruncPr's rounding draws differ from running
        the ops one by one.  MOOSEX_MERGE_ROUNDS=0 disables it."""
        def key(o):
            if not isinstance(o.placement, ReplicatedPlacement) or len(o.inputs) != 1:
                return None
            if o.inputs[0] not in self.env:
                return None
            x = self._at_memo_put(o, self.env[o.inputs[0]])  # e.g. a host input shared
            if (x.kind != "tensor" or x.dtype is None or not x.dtype.is_fixed or x.is_host
                    or x.is_mir or not isinstance(x.v, fxp.RepFixed)
                    or not isinstance(x.plc, ReplicatedPlacement) or x.plc != o.placement):
                return None
            return (o.kind, o.placement, x.dtype, repr(sorted(o.attrs.items()))), x

        k0 = key(op)
        if k0 is None:
            return False
        group = [(op, k0[1])]
        for o in later:
            if len(group) >= limit:
                break
            if o.kind != op.kind or o.name in self.env:
                continue
            if self._table_handler(o) is not None:
                continue
            k = key(o)
            if k is not None and k[0] == k0[0]:
                group.append((o, k[1]))
        if len(group) == 1:
            return False
        for o, lv in self._merge_compute(op.kind, group):
            if self.on_op is not None and self.lanes is None:
                self.on_op()
            self.env[o.name] = lv
        return True

    def _merge_compute(self, kind, group):
        """One protocol run of ``kind`` over the concatenated inputs of ``group`` [(op,
        converted input)]: [(op, its output LV)]."""
        sess = self.sess
        flats, metas = [], []
        for _o, x in group:
            try:
                shp = tuple(fxp.shape_of(sess, x.v))
            except Exception:  # noqa: BLE001 - this process holds no share: all remote
                shp = None
            n = math.prod(shp) if shp is not None else 1
            flats.append(fxp.local(sess, x.v, "Reshape", shape=(n,)))
            metas.append((shp, n))
        fn = _MERGE_FNS[kind]
        out = []
        with span(f"op.{kind}.merged", n=len(group)):
            y = fn(sess, fxp.concat(sess, flats, 0))
            at = 0
            for (o, x), (shp, n) in zip(group, metas):
                part = fxp.local(sess, y, "Slice", slice=(at, at + n, None))
                at += n
                if shp is not None:
                    part = fxp.local(sess, part, "Reshape", shape=shp)
                out.append((o, LV(x.plc, "tensor", x.dtype, part)))
        return out

    # ------------------------------------------------------------------------
    # dialect-level operations (textual computations below the logical level)
    # ------------------------------------------------------------------------
    def _table_handler(self, op):
        """Ring-level operations on replicated / additive placements (and their Reveal to a
        host) through the declarative (op, placement, operand types) table of
        runtime/dispatch.py; None when no row matches (logical types never do)."""
        if op.sig is None or not any(t.name not in _LOGICAL_TY for t in op.sig.args):
            return None  # logical signatures: no table row (fast path, checked per op)
        from moose_amd.ir.computation import AdditivePlacement
        from moose_amd.runtime import dispatch

        plc = op.placement
        kind = ("rep" if isinstance(plc, ReplicatedPlacement) else
                "adt" if isinstance(plc, AdditivePlacement) else
                "host" if isinstance(plc, HostPlacement) and op.kind == "Reveal" else None)
        if kind is None or op.sig is None:
            return None
        args = [t.name for t in op.sig.args]
        if op.sig.variadic and args:
            args = args[:1] * max(1, len(op.inputs))
        k = dispatch.lookup(op.kind, kind, args)
        if k is None:
            return None
        fams = [dispatch.family(t) for t in args]

        def run(op, ins):
            vals = []
            for x, f in zip(ins, fams):
                if f.startswith("rep_"):
                    if not x.is_rep:
                        x = self.to_rep(x, plc)
                    vals.append(x.v.t if isinstance(x.v, RepFixed) else x.v)
                else:  # additive shares, public host operands
                    vals.append(x.v)
            out = k.fn(dispatch.Ctx(self.sess, op), *vals)
            return LV(plc, "tensor", None, out)

        return run

    def _dialect_handler(self, op):
        """Handler for an operator without a logical ``op_*`` method: replicated dialect
        protocols (Share/Reveal/TruncPr/Msb/BitDecompose/...) or, on a host, the host
        primitive itself -- the role of the reference's SyncSession dispatch tables
        for host and replicated placements (``execution/synchronous.rs:149-237``)."""
        if isinstance(op.placement, ReplicatedPlacement) and op.kind in _REP_DIALECT:
            return self._rep_dialect
        if isinstance(op.placement, HostPlacement):
            from moose_amd.runtime.prims import PRIMS

            if op.kind in PRIMS:
                return self._host_prim
        return None

    def _host_prim(self, op, ins):
        from moose_amd.runtime.graph_executor import _attr_value
        from moose_amd.runtime.graph_executor import prim_attrs

        host = op.placement.owner
        hp = HostPlacement(host)
        args = []
        for x in ins:
            x = self.to_host(x, host)
            args.append(x.v if x.kind in ("tensor", "shape") else self._plain(x))
        attrs = {k: _attr_value(v) for k, v in op.attrs.items()}
        out = self.sess.h(op.kind, host, *args, **prim_attrs(op, attrs, self.sess.device))
        ret = op.sig.ret.name
        if ret == "HostShape":
            return LV(hp, "shape", None, out)
        dtype = {"HostFloat64Tensor": T.FLOAT64, "HostFloat32Tensor": T.FLOAT32,
                 "HostBitTensor": None, "HostUint64Tensor": T.UINT64}.get(ret)
        if ins and ins[0].dtype is not None and ins[0].dtype.is_fixed and ret.startswith(
                "HostFixed"):
            dtype = ins[0].dtype
        return LV(hp, "tensor", dtype, out)

    def _rep_dialect(self, op, ins):
        plc = op.placement
        sess = self.sess
        kind = op.kind
        if kind == "Share":
            x = ins[0]
            if x.is_host and x.dtype is None:  # raw ring / bit tensor
                bits = getattr(x.v.v, "bits", None)
                return LV(plc, "tensor", None,
                          rep.share(sess, plc, x.v, kind="bool" if bits == 1 else "arith"))
            return self.to_rep(x, plc)
        xs = [self.to_rep(x, plc) for x in ins]
        ts = [x.v.t if isinstance(x.v, RepFixed) else x.v for x in xs]
        attrs = op.attrs
        if kind == "TruncPr":
            amount = int(attrs.get("amount", attrs.get("precision", 0)))
            t = rep.trunc_pr(sess, ts[0], amount)
            if isinstance(xs[0].v, RepFixed):
                f = xs[0].v
                return LV(plc, "tensor", xs[0].dtype, RepFixed(t, f.frac - amount, f.integ))
            return LV(plc, "tensor", None, t)
        fn = _REP_DIALECT[kind]
        if kind == "Shl":
            t = fn(sess, ts[0], int(attrs["amount"]))
        elif kind == "BitExtract":
            t = fn(sess, ts[0], int(attrs["bit_idx"]))
        elif kind == "Index":  # bit i of a replicated bit array (packed words here)
            t = fn(sess, ts[0], int(attrs["index"]))
        elif kind == "RingInject":
            t = rep.shl(sess, fn(sess, ts[0], int(attrs.get("ring_bits", 0)) or
                                 (128 if "128" in op.sig.ret.name else 64)),
                        int(attrs.get("bit_idx", 0)))
        else:
            t = fn(sess, *ts)
        return LV(plc, "tensor", None, t)

    # ------------------------------------------------------------------------
    # SPMD: operations placed on other parties
    # ------------------------------------------------------------------------
    def _foreign_op(self, op, ins, me):
        """This process does not own ``op``'s placement.  It takes part only in moving
        its own operands there (sharing a host input, revealing a share, ...), in the
        order the owners' handler converts them, and keeps a typed placeholder."""
        for x in ins:
            if me in _owners(x.plc) and x.kind in ("tensor", "shape"):
                self.at(op, x)
        return self._placeholder(op)

    def _placeholder(self, op) -> LV:
        from moose_amd.parallel.spmd import Remote
        from moose_amd.runtime.session import PV

        plc = op.placement
        ret = op.sig.ret
        name = ret.name
        kind = ("shape" if "Shape" in name else "string" if "String" in name
                else "unit" if name == "Unit" else "tensor")
        dtype = self._ret_dtype(op) if kind == "tensor" else None
        bits = None
        if dtype is not None:
            bits = (dtype.ring_bits if dtype.is_fixed else 1 if dtype.kind == "Bool"
                    else 64 if dtype.kind == "Uint64" else None)
        if isinstance(plc, HostPlacement):
            return LV(plc, kind, dtype, HV(plc.owner, Remote(bits)))
        if isinstance(plc, ReplicatedPlacement) and kind == "tensor" and bits is not None:
            rkind = "bool" if bits == 1 else "arith"
            t = rep.RepTensor(plc, bits, rkind, PV(plc, Remote(bits)), PV(plc, Remote(bits)))
            if dtype.is_fixed:
                t = RepFixed(t, dtype.fractional_precision, dtype.integral_precision)
            return LV(plc, kind, dtype, t)
        return LV(plc, kind, dtype, MV(plc, Remote(bits)))

    # ------------------------------------------------------------------------
    # dtype helpers
    # ------------------------------------------------------------------------
    def _dtype(self, d: T.TensorDType) -> T.TensorDType:
        if d is not None and d.kind == "Fixed128" and self.fixed_ring == 64:
            return T.TensorDType("Fixed64", d.integral_precision, d.fractional_precision)
        return d

    def _ret_dtype(self, op):
        return self._dtype(op.sig.ret.dtype) if op.sig.ret.name == "Tensor" else None

    # ------------------------------------------------------------------------
    # placement conversions
    # ------------------------------------------------------------------------
    def to_host(self, x: LV, host: str) -> LV:
        sess = self.sess
        hp = HostPlacement(host)
        if x.is_host:
            if x.host == host:
                return x
            return LV(hp, x.kind, x.dtype, sess.move(x.v, host))
        if x.is_rep and isinstance(x.v, MV):
            return LV(hp, x.kind, x.dtype, HV(host, x.v.v))
        if x.is_mir:
            return LV(hp, x.kind, x.dtype, HV(host, x.v.v))
        if x.is_rep:
            if x.kind != "tensor":
                return LV(hp, x.kind, x.dtype, HV(host, x.v))
            if isinstance(x.v, RepFixed):
                ring = rep.reveal(sess, x.v.t, host)
                return LV(hp, "tensor", x.dtype, ring)
            opened = rep.reveal(sess, x.v, host)
            if x.dtype is None:  # raw ring / bit sharing (dialect-level Reveal)
                return LV(hp, "tensor", None, opened)
            if x.dtype.kind == "Bool":
                return LV(hp, "tensor", x.dtype, sess.h("ToBool", host, opened))
            if x.dtype.kind == "Uint64":
                return LV(hp, "tensor", x.dtype, sess.h("RingToInt", host, opened))
            return LV(hp, "tensor", x.dtype, opened)
        raise MooseRuntimeError(f"cannot move {x} to host {host}")

    def to_rep(self, x: LV, plc: ReplicatedPlacement) -> LV:
        if x.is_rep and x.plc == plc:
            return x
        if x.kind != "tensor":
            if x.kind == "shape":
                return LV(plc, "shape", None, self._plain(x))
            return x
        if x.is_mir or (x.is_rep and isinstance(x.v, MV)):
            return LV(plc, "tensor", x.dtype, MV(x.plc, x.v.v))
        if x.is_rep:  # another replicated placement: reveal then re-share
            x = self.to_host(x, plc.owners[0])
        d = x.dtype
        sess = self.sess
        if d.is_fixed:
            t = rep.share(sess, plc, x.v)
            return LV(plc, "tensor", d, RepFixed(t, d.fractional_precision, d.integral_precision))
        if d.kind == "Bool":
            bits = sess.h("FromBool", x.host, x.v)
            return LV(plc, "tensor", d, rep.share(sess, plc, bits, kind="bool"))
        if d.kind == "Uint64":
            ring = sess.h("IntToRing", x.host, x.v)
            return LV(plc, "tensor", d, rep.share(sess, plc, ring))
        raise MooseRuntimeError(
            f"cannot secret-share a {d} tensor; cast it to a fixed-point dtype first"
        )

    def to_mir(self, x: LV, plc: Mirrored3Placement) -> LV:
        if x.is_mir and x.plc == plc:
            return x
        if x.is_rep and isinstance(x.v, MV):
            return LV(plc, x.kind, x.dtype, MV(plc, x.v.v))
        h = self.to_host(x, plc.owners[0]) if not x.is_host else x
        return LV(plc, h.kind, h.dtype, self.sess.mirror(h.v, plc))

    def _plain(self, x: LV):
        """Python/plaintext value of a non-secret LV (shapes, strings, scalars)."""
        v = x.v
        if isinstance(v, (HV, MV)):
            v = v.v
        const = getattr(v, "const", None)  # symbolic value with a statically known value
        return const if const is not None else v

    @property
    def symbolic(self) -> bool:
        return getattr(self.sess, "symbolic", False)

    def _public(self, x: LV):
        return x.v.v if isinstance(x.v, MV) else None

    def _at_memo_put(self, op, x: LV) -> LV:
        """``at`` for the batching probe: the converted value (e.g. a fresh sharing of a host
        input) is kept so that executing ``op`` later reuses it instead of sharing again."""
        memo = self.__dict__.setdefault("_at_memo", {})
        hit = memo.get((id(x), op.placement))
        if hit is not None and hit[0] is x:
            return hit[1]
        conv = self.at(op, x)
        if conv is not x:
            # with lanes, the op that reuses it may run on another stream: it waits on this
            ev = self.lanes.mark() if self.lanes is not None else None
            memo[(id(x), op.placement)] = (x, conv, ev)
        return conv

    def at(self, op, x: LV) -> LV:
        plc = op.placement
        pre = self.__dict__.get("_lockstep_pre")
        if pre:  # converted for this op before its lockstep group started (_lockstep)
            hit = pre.pop((op.name, id(x)), None)
            if hit is not None and hit[0] is x:
                return hit[1]
        memo = self.__dict__.get("_at_memo")
        if memo:
            hit = memo.pop((id(x), plc), None)
            if hit is not None and hit[0] is x:
                if hit[2] is not None and self.lanes is not None:
                    self.lanes.wait_mark(hit[2], hit[1])
                return hit[1]
        if isinstance(plc, HostPlacement):
            return self.to_host(x, plc.owner)
        if isinstance(plc, ReplicatedPlacement):
            return self.to_rep(x, plc)
        if isinstance(plc, Mirrored3Placement):
            return self.to_mir(x, plc)
        raise MooseRuntimeError(f"unsupported placement {plc}")

    # ------------------------------------------------------------------------
    # IO
    # ------------------------------------------------------------------------
    def _host_value_from_python(self, host, value, want: T.Ty):
        sess = self.sess
        hp = HostPlacement(host)
        if isinstance(value, str):
            return LV(hp, "string", None, HV(host, value))
        if isinstance(value, (tuple, list)) and want is not None and want.name in ("HostShape", "Shape"):
            return LV(hp, "shape", None, HV(host, tuple(value)))
        if isinstance(value, float) and not isinstance(value, np.ndarray):
            if want is None or want.name != "Tensor":
                return LV(hp, "float", None, HV(host, value))
        if isinstance(value, int) and not isinstance(value, bool):
            if want is None or want.name != "Tensor":
                return LV(hp, "int", None, HV(host, value))
        if isinstance(value, torch.Tensor):  # device-resident argument (no host copy)
            t = value.to(sess.device)
            dtype = getattr(value, "_moose_dtype", None) or {
                torch.float64: T.FLOAT64, torch.float32: T.FLOAT32,
                torch.bool: T.BOOL}.get(t.dtype, T.UINT64)
        else:
            arr = np.asarray(value)
            dtype = dtype_of_numpy(arr)
            t = numpy_to_torch(arr, sess.device)
        lv = LV(hp, "tensor", dtype, HV(host, t))
        if want is not None and want.name == "Tensor" and want.dtype.kind not in ("Unknown",):
            wd = self._dtype(want.dtype)
            if wd != dtype:
                lv = self._cast_host(lv, wd)
        return lv

    def op_Reveal(self, op, ins):
        return self.to_host(ins[0], op.placement.owner)

    # mirrored / fixed-point dialect conversions (reference kernels/conversion.rs)
    def op_Mirror(self, op, ins):
        return self.to_mir(ins[0], op.placement)

    def op_Demirror(self, op, ins):
        return self.to_host(ins[0], op.placement.owner)

    def op_FixedpointEncode(self, op, ins):
        kind = "Fixed64" if "64" in op.sig.ret.name else "Fixed128"
        if self.fixed_ring == 64:
            kind = "Fixed64"
        d = T.TensorDType(kind, int(op.attrs.get("integral_precision", 0)),
                          int(op.attrs["fractional_precision"]))
        return self.at(op, self._cast_host(self.to_host(ins[0], _owners(op.placement)[0]), d))

    def op_FixedpointDecode(self, op, ins):
        want = T.FLOAT32 if "32" in op.sig.ret.name else T.FLOAT64
        return self.at(op, self._cast_host(self.to_host(ins[0], _owners(op.placement)[0]), want))

    def op_Pow2(self, op, ins):
        plc = op.placement
        x = self.to_rep(ins[0], plc) if isinstance(plc, ReplicatedPlacement) else ins[0]
        if not (x.is_rep and isinstance(x.v, RepFixed)):
            raise MooseRuntimeError("Pow2 is defined on replicated fixed-point tensors")
        return LV(plc, "tensor", x.dtype, fxp.exp2(self.sess, x.v))

    def op_Input(self, op, ins):
        name = op.attrs.get("arg_name") or op.name
        if self.symbolic:
            return self._symbolic_input(op, name)
        rname = op.sig.ret.name
        if rname in ("AesKey", "HostAesKey", "ReplicatedAesKey"):
            from moose_amd.protocols import aes

            return aes.key_input(self, op, name)
        if rname in ("AesTensor", "Fixed128AesTensor", "HostFixed128AesTensor"):
            from moose_amd.protocols import aes

            return aes.tensor_input(self, op, name)
        plc = op.placement
        if isinstance(plc, ReplicatedPlacement) and (
                rname in shares.REP_TYPES or (name not in self.arguments and any(
                    shares.share_name(name, r, i) in self.arguments
                    for i, r in enumerate(plc.owners)))):
            return self._preshared_input(op, name)
        if name not in self.arguments:
            raise MooseRuntimeError(f"missing argument {name}")
        host = plc.owner if isinstance(plc, HostPlacement) else plc.owners[0]
        lv = self._host_value_from_python(host, self.arguments[name], op.sig.ret)
        return lv if isinstance(plc, HostPlacement) else self.at(op, lv)

    def _rep_type_info(self, op, meta=None):
        """(bits, kind, dtype) of a replicated Input/Load from its type (or saved meta)."""
        ret = op.sig.ret
        if ret.name in shares.REP_TYPES:
            bits, kind, dtype = shares.REP_TYPES[ret.name]
            return bits, kind, (meta or {}).get("dtype", dtype)
        if meta is not None:
            return meta["bits"], meta["kind"], meta.get("dtype")
        d = self._dtype(ret.dtype) if ret.name == "Tensor" else T.UNKNOWN_DTYPE
        if d.is_fixed:
            return d.ring_bits, "arith", d
        if d.kind == "Bool":
            return 1, "bool", d
        if d.kind == "Uint64":
            return 64, "arith", d
        raise MooseRuntimeError(f"{op.name}: cannot infer the share type of {ret}")

    def _rep_lv(self, plc, t, dtype):
        if dtype is not None and dtype.is_fixed:
            return LV(plc, "tensor", dtype, RepFixed(t, dtype.fractional_precision,
                                                     dtype.integral_precision))
        return LV(plc, "tensor", dtype, t)

    def _preshared_input(self, op, name):
        """Replicated Input from pre-shared ``name/<role>/share<i>`` arguments."""
        plc = op.placement
        bits, kind, dtype = self._rep_type_info(op)

        def lookup(p, i):
            k = shares.share_name(name, plc.owners[p], i)
            if k not in self.arguments:
                raise MooseRuntimeError(f"missing pre-shared argument {k}")
            return self.arguments[k]

        t = shares.rep_from_components(self.sess, plc, bits, kind, lookup)
        return self._rep_lv(plc, t, dtype)

    def _save_shares(self, plc, key, val: LV):
        """Each party stores its own pair of shares in its own storage."""
        v = val.v
        if isinstance(v, MV):
            raise MooseRuntimeError("saving a public value on a replicated placement; "
                                    "save it on a host instead")
        t = v.t if isinstance(v, RepFixed) else v
        dtype = val.dtype
        if isinstance(v, RepFixed) and (dtype is None or not dtype.is_fixed):
            dtype = T.TensorDType("Fixed64" if t.bits == 64 else "Fixed128", v.integ, v.frac)
        comps = shares.rep_components(self.sess, t)
        for p, c in enumerate(comps):
            if c is None:
                continue
            role = plc.owners[p]
            store = self.storage.setdefault(role, {})
            store[shares.share_name(key, role, p)] = shares.ring_to_python(c[0])
            store[shares.share_name(key, role, (p + 1) % 3)] = shares.ring_to_python(c[1])
            store[shares.meta_name(key, role)] = shares.meta_json(t.bits, t.kind, dtype)

    def _load_shares(self, op, key):
        plc = op.placement
        me = getattr(self.sess, "me", None)
        mine = [r for r in plc.owners if me is None or r == me]
        meta_s = self.storage.get(mine[0], {}).get(shares.meta_name(key, mine[0]))
        if meta_s is None:
            raise MooseRuntimeError(f"no share checkpoint {key!r} in storage of {mine[0]}")
        bits, kind, dtype = self._rep_type_info(op, shares.parse_meta(meta_s))

        def lookup(p, i):
            role = plc.owners[p]
            k = shares.share_name(key, role, i)
            store = self.storage.get(role, {})
            if k not in store:
                raise MooseRuntimeError(f"key {k!r} not found in storage of {role}")
            return store[k]

        t = shares.rep_from_components(self.sess, plc, bits, kind, lookup)
        return self._rep_lv(plc, t, dtype)

    def _const_key(self, c, host, want):
        """Cache key of a small numeric tensor constant on a device session: its bytes,
        dtype, shape, kind, the wanted type, host and device (the value itself, so a key
        never outlives what it names).  None: not cached."""
        dev = getattr(self.sess, "device", None)
        if self.symbolic or dev is None or dev.type != "cuda" or c.kind in (
                "HostShape", "HostString", "HostRing64Tensor", "HostRing128Tensor"):
            return None
        try:
            arr = np.asarray(c.value)
        except Exception:  # noqa: BLE001 - anything unusual stays uncached
            return None
        if arr.dtype == object or arr.nbytes > (1 << 16) or (
                c.kind in ("Float32", "Float64") and want.name != "Tensor"):
            return None
        return (c.kind, arr.dtype.str, arr.shape, arr.tobytes(), repr(want), host, str(dev))

    def op_Constant(self, op, ins):
        c: Constant = op.attrs["value"]
        plc = op.placement
        host = plc.owner if isinstance(plc, HostPlacement) else plc.owners[0]
        want = op.sig.ret
        hp = HostPlacement(host)
        key = self._const_key(c, host, want)
        hit = _CONST_LV.get(key) if key is not None else None
        if hit is not None:  # uploaded once: no host->device copy per evaluation
            lv = hit
        elif c.kind == "HostShape":
            lv = LV(hp, "shape", None, HV(host, tuple(c.value)))
        elif c.kind == "HostString":
            lv = LV(hp, "string", None, HV(host, c.value))
        elif c.kind in ("Float32", "Float64"):
            lv = self._host_value_from_python(host, np.array(c.value, dtype=np.float64)
                                              if want.name == "Tensor" else float(c.value), want)
        elif c.kind in ("HostRing64Tensor", "HostRing128Tensor"):
            bits = 64 if "64" in c.kind else 128
            lv = LV(hp, "tensor", None, HV(host, R.from_ints(c.value, bits, self.sess.device)))
        else:
            arr = np.asarray(c.value)
            lv = self._host_value_from_python(host, arr, want)
        if (key is not None and hit is None and isinstance(lv.v, HV)
                and isinstance(lv.v.v, torch.Tensor) and lv.v.v.is_cuda
                and not torch.cuda.is_current_stream_capturing()):
            if len(_CONST_LV) < 1024:  # public constants are never written
                if _lanes.ACTIVE or R.SHARED_STREAMS:  # other streams read it next
                    torch.cuda.current_stream(lv.v.v.device).synchronize()
                with _CONST_LOCK:
                    # parties on threads may make the same constant at once: the first in
                    # stays cached and is used; an id is registered only for a tensor the
                    # cache keeps alive (a dropped one's id could return as another's)
                    kept = _CONST_LV.setdefault(key, lv)
                    if kept is lv:
                        R.CONST_IDS.add(id(lv.v.v))
                lv = kept
        if isinstance(plc, HostPlacement):
            return lv
        # constants on replicated / mirrored placements are public
        if isinstance(plc, ReplicatedPlacement):
            return LV(plc, lv.kind, lv.dtype, MV(plc, lv.v.v))
        return LV(plc, lv.kind, lv.dtype, MV(plc, lv.v.v))

    def op_Output(self, op, ins):
        x = ins[0]
        plc = op.placement
        if isinstance(plc, HostPlacement):
            x = self.to_host(x, plc.owner)
        elif x.kind == "tensor":
            # outputs pinned to a replicated / mirrored placement open to its first owner
            x = self.to_host(x, plc.owners[0])
        tag = op.attrs.get("tag") or op.name
        if self.symbolic:
            sess = self.sess
            v = x.v.v if isinstance(x.v, (HV, MV)) else x.v
            sess.output(x.plc.owner if x.is_host else plc.owners[0], tag,
                        sess.lit(x.plc.owner if x.is_host else plc.owners[0], v))
        self.outputs[tag] = x
        return x

    def _symbolic_input(self, op, name):
        """Lowering: an Input op of the lowered graph with the shape from ``arg_specs``."""
        from moose_amd.compiler.symbolic import ring_ty

        spec = self.arg_specs.get(name) if getattr(self, "arg_specs", None) else None
        # no spec: shape-polymorphic lowering -- the value's shape is unknown (None) and
        # every protocol step that needs it reads it at run time through a Shape op
        # (reference execution/symbolic.rs:400-435); the dtype comes from the signature
        shape, dtype = spec if spec is not None else (None, None)
        plc = op.placement
        host = plc.owner if isinstance(plc, HostPlacement) else plc.owners[0]
        hp = HostPlacement(host)
        want = op.sig.ret
        d = dtype if dtype is not None else (want.dtype if want.name == "Tensor" else T.FLOAT64)
        d = self._dtype(d)
        if d.is_fixed:
            ty, bits = ring_ty(d.ring_bits), d.ring_bits
        else:
            ty, bits = T.Ty({"Float64": "HostFloat64Tensor", "Float32": "HostFloat32Tensor",
                             "Bool": "HostBitTensor", "Uint64": "HostUint64Tensor"}[d.kind]), None
        lv = LV(hp, "tensor", d, HV(host, self.sess.input(host, name, ty, shape, bits)))
        if want.name == "Tensor" and want.dtype.kind != "Unknown":
            wd = self._dtype(want.dtype)
            if wd != d:
                lv = self._cast_host(lv, wd)
        return lv if isinstance(plc, HostPlacement) else self.at(op, lv)

    def op_Identity(self, op, ins):
        return self.at(op, ins[0])

    def op_Save(self, op, ins):
        key, val = ins
        k = self._plain(key)
        if isinstance(op.placement, ReplicatedPlacement):
            plc = op.placement
            self._save_shares(plc, k, self.to_rep(val, plc))
            return LV(plc, "unit", None, MV(plc, None))
        host = op.placement.owner
        val = self.to_host(val, host)
        if self.storage_tap is not None:  # a capture: stored after each replay
            self.storage_tap.record_save(host, k, self, val)
        elif self.sess.materialized(val.v):
            self.storage.setdefault(host, {})[k] = self.to_numpy(val)
        return LV(op.placement, "unit", None, HV(host, None))

    def op_Load(self, op, ins):
        key, query = ins
        k = self._plain(key)
        if isinstance(op.placement, ReplicatedPlacement):
            return self._load_shares(op, k)
        host = op.placement.owner
        if self.storage_tap is not None:  # a capture: a static buffer refreshed per replay
            return self._host_value_from_python(host, self.storage_tap.load(host, k),
                                                op.sig.ret)
        store = self.storage.get(host, {})
        if k not in store:
            from moose_amd.utils import storage as st

            value = st.load_from_path(k, self._plain(query)) if st.looks_like_path(k) else None
            if value is None:
                raise MooseRuntimeError(f"key {k!r} not found in storage of {host}")
        else:
            value = store[k]
        return self._host_value_from_python(host, value, op.sig.ret)

    # ------------------------------------------------------------------------
    # materialisation
    # ------------------------------------------------------------------------
    def to_numpy(self, x: LV):
        v = self._plain(x)
        if x.kind != "tensor":
            return v
        if isinstance(v, R.RT):
            if x.dtype is not None and x.dtype.is_fixed:
                return R.decode(v, x.dtype.fractional_precision).cpu().numpy()
            return R.to_ints(v)
        t = v.detach().cpu()
        if x.dtype is not None and x.dtype.kind == "Uint64":
            return t.numpy().view(np.uint64)
        return t.numpy()

    # ------------------------------------------------------------------------
    # casts
    # ------------------------------------------------------------------------
    def _cast_host(self, x: LV, target: T.TensorDType) -> LV:
        sess, host = self.sess, x.host
        src = x.dtype
        if src == target:
            return x
        if target.is_fixed:
            bits = target.ring_bits
            if src.is_fixed:
                v = x.v
                df = target.fractional_precision - src.fractional_precision
                if src.ring_bits != bits:
                    v = sess.h("RingCast", host, v, bits=bits)
                if df > 0:
                    v = sess.h("Shl", host, v, amount=df)
                elif df < 0:
                    v = sess.h("Sar", host, v, amount=-df)
                return LV(x.plc, "tensor", target, v)
            f = sess.h("Cast", host, x.v, dtype=torch.float64)
            return LV(x.plc, "tensor", target,
                      sess.h("RingFixedpointEncode", host, f,
                             scaling_exp=target.fractional_precision, bits=bits))
        if src is not None and src.is_fixed:
            f = sess.h("RingFixedpointDecode", host, x.v, scaling_exp=src.fractional_precision)
            if target.kind == "Float64":
                return LV(x.plc, "tensor", target, f)
            x = LV(x.plc, "tensor", T.FLOAT64, f)
            src = T.FLOAT64
        if src is None:  # raw ring tensor
            raise MooseRuntimeError("cannot cast a raw ring tensor")
        return LV(x.plc, "tensor", target, sess.h("Cast", host, x.v, dtype=torch_dtype_of(target)))

    def op_Cast(self, op, ins):
        target = self._ret_dtype(op)
        x = self.at(op, ins[0])
        if x.is_host:
            return self._cast_host(x, target)
        if x.is_rep and isinstance(x.v, MV):
            h = self._cast_host(LV(HostPlacement(op.placement.owners[0]), x.kind, x.dtype,
                                   HV(op.placement.owners[0], x.v.v)), target)
            return LV(x.plc, "tensor", target, MV(x.plc, h.v.v))
        if x.is_rep:
            src = x.dtype
            if src.is_fixed and target.is_fixed:
                return LV(x.plc, "tensor", target, fxp.cast(self.sess, x.v, target))
            if src.kind == "Bool" and target.is_fixed:
                t = rep.b2a(self.sess, x.v, target.ring_bits)
                f = target.fractional_precision
                t = rep.shl(self.sess, t, f) if f else t
                return LV(x.plc, "tensor", target,
                          RepFixed(t, f, target.integral_precision))
            raise MooseRuntimeError(f"replicated cast {src} -> {target} not supported")
        if x.is_mir:
            h = self._cast_host(LV(HostPlacement(x.plc.owners[0]), x.kind, x.dtype,
                                   HV(x.plc.owners[0], x.v.v)), target)
            return LV(x.plc, "tensor", target, MV(x.plc, h.v.v))
        raise MooseRuntimeError("bad cast")

    # ------------------------------------------------------------------------
    # arithmetic
    # ------------------------------------------------------------------------
    def _binary(self, op, ins, kind):
        x, y = (self.at(op, v) for v in ins)
        if x.kind != "tensor" or y.kind != "tensor":
            return self._scalar_binary(op, x, y, kind)
        dtype = x.dtype if x.dtype is not None else y.dtype
        if x.is_host:
            return self._host_binary(op, x, y, kind, dtype)
        if x.is_mir:
            return self._mir_binary(op, x, y, kind, dtype)
        return self._rep_binary(op, x, y, kind, dtype)

    def _scalar_binary(self, op, x, y, kind):
        a, b = self._plain(x), self._plain(y)
        f = {"Add": lambda: a + b, "Sub": lambda: a - b, "Mul": lambda: a * b,
             "Div": lambda: a / b}[kind]
        return LV(x.plc, x.kind, None, HV(getattr(x.plc, "owner", None), f()))

    def _host_binary(self, op, x, y, kind, dtype):
        sess, host = self.sess, x.host
        if dtype.is_fixed:
            f = dtype.fractional_precision
            if kind in ("Add", "Sub"):
                return LV(x.plc, "tensor", dtype, sess.h(kind, host, x.v, y.v))
            if kind in ("Mul", "Dot"):
                z = sess.h(kind, host, x.v, y.v)
                return LV(x.plc, "tensor", dtype, sess.h("Sar", host, z, amount=f))
            if kind == "Div":
                xf = sess.h("RingFixedpointDecode", host, x.v, scaling_exp=f)
                yf = sess.h("RingFixedpointDecode", host, y.v, scaling_exp=f)
                q = sess.h("Div", host, xf, yf)
                return LV(x.plc, "tensor", dtype, sess.h("RingFixedpointEncode", host, q,
                                                         scaling_exp=f, bits=dtype.ring_bits))
        if kind in ("Less", "Greater"):
            return LV(x.plc, "tensor", T.BOOL, sess.h(kind, host, x.v, y.v))
        if kind in ("And", "Or"):
            return LV(x.plc, "tensor", dtype, sess.h(kind, host, x.v, y.v))
        return LV(x.plc, "tensor", dtype, sess.h(kind, host, x.v, y.v))

    def _mir_binary(self, op, x, y, kind, dtype):
        hx = LV(HostPlacement(x.plc.owners[0]), "tensor", x.dtype, HV(x.plc.owners[0], x.v.v))
        hy = LV(HostPlacement(x.plc.owners[0]), "tensor", y.dtype, HV(x.plc.owners[0], y.v.v))
        r = self._host_binary(op, hx, hy, kind, dtype)
        return LV(x.plc, "tensor", r.dtype, MV(x.plc, r.v.v))

    def _broadcast_secret(self, x, y, px, py, kind=None):
        """Numpy-broadcast the secret operand(s) of an elementwise op to the common shape.

        Shares carry a leading party axis (stacked) or live per process (SPMD), so rank
        differences must be resolved on the logical shapes before the share-wise kernels
        (e.g. a shared scalar learning rate times a (100, 1) gradient)."""
        def shape(v, pub):
            if pub is not None:
                s = getattr(pub, "shape", None)
                return tuple(s) if s is not None else ()
            try:
                s = fxp.shape_of(self.sess, v.v)
            except RuntimeError:
                return None
            return None if s is None or any(d is None for d in s) else tuple(s)

        sx, sy = shape(x, px), shape(y, py)
        if sx is None or sy is None or sx == sy:
            return x, y
        target = tuple(np.broadcast_shapes(sx, sy))
        if (BCAST_IN_KERNEL and kind in ("Add", "Sub", "Mul") and px is None and py is None
                and getattr(self.sess, "party_jobs", None) is not None
                and ((math.prod(sx) == 1 and sy == target)
                     or (math.prod(sy) == 1 and sx == target))):
            # a per-party session broadcasts a one-element operand inside its kernels
            # (share-wise add / sub: ring.binary2; mul: a stride-0 row of the batched tail,
            # rep.mul_trunc): no materialised copy
            return x, y
        if px is None and sx != target:
            x = LV(x.plc, x.kind, x.dtype, fxp.broadcast_to(self.sess, x.v, target))
        if py is None and sy != target:
            y = LV(y.plc, y.kind, y.dtype, fxp.broadcast_to(self.sess, y.v, target))
        return x, y

    def _rep_binary(self, op, x, y, kind, dtype):
        sess = self.sess
        px, py = self._public(x), self._public(y)
        if px is not None and py is not None:
            h = self._mir_binary(op, LV(x.plc, "tensor", x.dtype, MV(x.plc, px)),
                                 LV(x.plc, "tensor", y.dtype, MV(x.plc, py)), kind, dtype)
            return LV(x.plc, "tensor", h.dtype, MV(x.plc, h.v.v))
        if kind != "Dot":
            x, y = self._broadcast_secret(x, y, px, py, kind)
        if kind in ("Less", "Greater"):
            a, b = x, y
            return LV(x.plc, "tensor", T.BOOL, fxp.compare(sess, kind, a.v, b.v, px, py))
        if kind in ("And", "Or"):
            if px is not None or py is not None:
                raise MooseRuntimeError("boolean ops with public operands not supported")
            if kind == "And":
                return LV(x.plc, "tensor", T.BOOL, rep.and_(sess, x.v, y.v))
            # a | b = a ^ b ^ (a & b)
            return LV(x.plc, "tensor", T.BOOL,
                      rep.xor(sess, rep.xor(sess, x.v, y.v), rep.and_(sess, x.v, y.v)))
        if dtype.kind == "Uint64":
            return LV(x.plc, "tensor", dtype, fxp.ring_binary(sess, kind, x.v, y.v, px, py))
        if not dtype.is_fixed:
            raise MooseRuntimeError(f"replicated {kind} on {dtype}")
        f = dtype.fractional_precision
        if kind == "Add":
            r = fxp.add(sess, x.v, y.v, px, py)
        elif kind == "Sub":
            r = fxp.sub(sess, x.v, y.v, px, py)
        elif kind == "Mul":
            r = fxp.mul(sess, x.v, y.v, px, py, f)
        elif kind == "Dot":
            r = fxp.dot(sess, x.v, y.v, px, py, f)
        elif kind == "Div":
            r = fxp.div(sess, x.v, y.v, px, py)
        else:
            raise MooseRuntimeError(kind)
        return LV(x.plc, "tensor", dtype, r)

    def op_Add(self, op, ins):
        return self._binary(op, ins, "Add")

    def op_Sub(self, op, ins):
        return self._binary(op, ins, "Sub")

    def op_Mul(self, op, ins):
        return self._binary(op, ins, "Mul")

    def op_Dot(self, op, ins):
        return self._binary(op, ins, "Dot")

    def op_Div(self, op, ins):
        return self._binary(op, ins, "Div")

    def op_Less(self, op, ins):
        return self._binary(op, ins, "Less")

    def op_Greater(self, op, ins):
        return self._binary(op, ins, "Greater")

    def op_And(self, op, ins):
        return self._binary(op, ins, "And")

    def op_Or(self, op, ins):
        return self._binary(op, ins, "Or")

    def op_AddN(self, op, ins):
        if (len(ins) > 2 and all(x.is_rep and isinstance(x.v, RepFixed) for x in ins)
                and len({(x.v.frac, x.dtype) for x in ins}) == 1):
            t = rep.add_n(self.sess, [x.v.t for x in ins])
            v = ins[0].v
            return LV(ins[0].plc, "tensor", ins[0].dtype, RepFixed(t, v.frac, v.integ))
        acc = ins[0]
        for x in ins[1:]:
            acc = self._binary(op, [acc, x], "Add")
        return acc

    # ------------------------------------------------------------------------
    # unary math
    # ------------------------------------------------------------------------
    def _host_float_unary(self, op, x, prim, **attrs):
        """Host math; fixed-point host tensors go through float64."""
        sess, host = self.sess, x.host
        d = x.dtype
        if d is not None and d.is_fixed:
            f = sess.h("RingFixedpointDecode", host, x.v, scaling_exp=d.fractional_precision)
            r = sess.h(prim, host, f, **attrs)
            if prim == "Argmax":
                return LV(x.plc, "tensor", T.UINT64, r)
            return LV(x.plc, "tensor", d, sess.h("RingFixedpointEncode", host, r,
                                                 scaling_exp=d.fractional_precision,
                                                 bits=d.ring_bits))
        r = sess.h(prim, host, x.v, **attrs)
        return LV(x.plc, "tensor", T.UINT64 if prim == "Argmax" else d, r)

    def _unary(self, op, ins, prim, rep_fn, **attrs):
        x = self.at(op, ins[0])
        if x.is_host:
            return self._host_float_unary(op, x, prim, **attrs)
        if x.is_mir or (x.is_rep and isinstance(x.v, MV)):
            h = self._host_float_unary(op, LV(HostPlacement(x.plc.owners[0]), x.kind, x.dtype,
                                              HV(x.plc.owners[0], x.v.v)), prim, **attrs)
            return LV(x.plc, "tensor", h.dtype, MV(x.plc, h.v.v))
        return rep_fn(x)

    def _rep_fixed_unary(self, fn, out_dtype=None):
        def apply(x):
            if not x.dtype.is_fixed:
                raise MooseRuntimeError(f"{fn.__name__} expects a fixed-point tensor, got {x.dtype}")
            return LV(x.plc, "tensor", out_dtype or x.dtype, fn(self.sess, x.v))

        return apply

    def op_Exp(self, op, ins):
        return self._unary(op, ins, "Exp", self._rep_fixed_unary(fxp.exp))

    def op_Log(self, op, ins):
        return self._unary(op, ins, "Log", self._rep_fixed_unary(fxp.log))

    def op_Log2(self, op, ins):
        return self._unary(op, ins, "Log2", self._rep_fixed_unary(fxp.log2))

    def op_Sqrt(self, op, ins):
        return self._unary(op, ins, "Sqrt", self._rep_fixed_unary(fxp.sqrt))

    def op_Sigmoid(self, op, ins):
        return self._unary(op, ins, "Sigmoid", self._rep_fixed_unary(fxp.sigmoid))

    def op_Relu(self, op, ins):
        return self._unary(op, ins, "Relu", self._rep_fixed_unary(fxp.relu))

    def op_Abs(self, op, ins):
        return self._unary(op, ins, "Abs", self._rep_fixed_unary(fxp.abs_))

    def op_Neg(self, op, ins):
        return self._unary(op, ins, "Neg", self._rep_fixed_unary(fxp.neg))

    def op_Softmax(self, op, ins):
        ax, up = op.attrs["axis"], op.attrs["upmost_index"]
        return self._unary(op, ins, "Softmax",
                           self._rep_fixed_unary(lambda s, v: fxp.softmax(s, v, ax, up)),
                           axis=ax, upmost_index=up)

    def op_Argmax(self, op, ins):
        ax, up = op.attrs["axis"], op.attrs["upmost_index"]

        def rep_fn(x):
            return LV(x.plc, "tensor", T.UINT64, fxp.argmax(self.sess, x.v, ax, up))

        return self._unary(op, ins, "Argmax", rep_fn, axis=ax, upmost_index=up)

    def op_Maximum(self, op, ins):
        xs = [self.at(op, v) for v in ins]
        if xs[0].is_host:
            r = self.sess.h("Maximum", xs[0].host, *[x.v for x in xs])
            return LV(xs[0].plc, "tensor", xs[0].dtype, r)
        return LV(xs[0].plc, "tensor", xs[0].dtype, fxp.maximum(self.sess, [x.v for x in xs]))

    def op_Inverse(self, op, ins):
        x = self.at(op, ins[0])
        if not x.is_host:
            raise MooseRuntimeError("Inverse is only supported on host placements")
        return self._host_float_unary(op, x, "Inverse")

    def op_Mux(self, op, ins):
        s, x, y = (self.at(op, v) for v in ins)
        if s.is_host:
            return LV(s.plc, "tensor", x.dtype, self.sess.h("Mux", s.host, s.v, x.v, y.v))
        # public (mirrored / constant) branches become trivial sharings (no messages)
        x, y = (v if not isinstance(v.v, MV) else self._share_public(v) for v in (x, y))
        if isinstance(s.v, MV):
            raise MooseRuntimeError("mux with a public selector on a replicated placement")
        xv, yv = x.v, y.v
        shp = fxp.shape_of(self.sess, s.v)
        xv, yv = (fxp.broadcast_to(self.sess, v, shp) for v in (xv, yv))
        return LV(s.plc, "tensor", x.dtype, fxp.mux(self.sess, s.v, xv, yv))

    # ------------------------------------------------------------------------
    # reductions
    # ------------------------------------------------------------------------
    def op_Sum(self, op, ins):
        x = self.at(op, ins[0])
        axis = op.attrs.get("axis")
        if x.is_host:
            return LV(x.plc, "tensor", x.dtype, self.sess.h("Sum", x.host, x.v, axis=axis))
        if isinstance(x.v, MV):
            return self._public_prim(x, "Sum", axis=axis)
        return LV(x.plc, "tensor", x.dtype, fxp.local(self.sess, x.v, "Sum", axis=axis))

    def op_Mean(self, op, ins):
        x = self.at(op, ins[0])
        axis = op.attrs.get("axis")
        if x.is_host:
            if x.dtype is not None and x.dtype.is_fixed:
                return self._host_float_unary(op, x, "Mean", axis=axis)
            return LV(x.plc, "tensor", x.dtype, self.sess.h("Mean", x.host, x.v, axis=axis))
        return LV(x.plc, "tensor", x.dtype, fxp.mean(self.sess, x.v, axis))

    # ------------------------------------------------------------------------
    # shape ops (share-wise on replicated values)
    # ------------------------------------------------------------------------
    def _public_prim(self, x, prim, *extra, **attrs):
        r = self.sess.h(prim, x.plc.owners[0], HV(x.plc.owners[0], x.v.v), *extra, **attrs)
        return LV(x.plc, x.kind, x.dtype, MV(x.plc, r.v))

    def _shape_op(self, op, x, prim, *extra, **attrs):
        x = self.at(op, x)
        if x.kind == "shape":
            return x
        if x.is_host:
            return LV(x.plc, "tensor", x.dtype, self.sess.h(prim, x.host, x.v, *extra, **attrs))
        if isinstance(x.v, MV):
            return self._public_prim(x, prim, *extra, **attrs)
        return LV(x.plc, "tensor", x.dtype, fxp.local(self.sess, x.v, prim, *extra, **attrs))

    def op_Transpose(self, op, ins):
        return self._shape_op(op, ins[0], "Transpose")

    def op_ExpandDims(self, op, ins):
        return self._shape_op(op, ins[0], "ExpandDims", axis=op.attrs["axis"])

    def op_Squeeze(self, op, ins):
        return self._shape_op(op, ins[0], "Squeeze", axis=op.attrs.get("axis"))

    def op_IndexAxis(self, op, ins):
        return self._shape_op(op, ins[0], "IndexAxis", axis=op.attrs["axis"],
                              index=op.attrs["index"])

    def op_AtLeast2D(self, op, ins):
        return self._shape_op(op, ins[0], "AtLeast2D",
                              to_column_vector=op.attrs["to_column_vector"])

    def op_Diag(self, op, ins):
        return self._shape_op(op, ins[0], "Diag")

    def op_Reshape(self, op, ins):
        shape = tuple(self._plain(ins[1]))
        return self._shape_op(op, ins[0], "Reshape", shape=shape)

    def op_Broadcast(self, op, ins):
        shape = tuple(self._plain(ins[1]))
        return self._shape_op(op, ins[0], "Broadcast", shape=shape)

    def op_Slice(self, op, ins):
        x = ins[0]
        sl = op.attrs["slice"]
        if x.kind == "shape":
            start, end, step = sl[0] if isinstance(sl, list) else sl
            v = tuple(self._plain(x))[start:end:step]
            return LV(x.plc if isinstance(op.placement, HostPlacement) else op.placement,
                      "shape", None, HV(getattr(op.placement, "owner", None), v)
                      if isinstance(op.placement, HostPlacement) else v)
        slices = sl if isinstance(sl, list) else [sl]
        py = [slice(a, b, c) for (a, b, c) in slices]
        return self._shape_op(op, x, "StridedSlice", slices=py)

    def op_Select(self, op, ins):
        # operands (index, x), as the reference's SelectOp (kernels/indexing.rs:60)
        idx, x = ins[0], ins[1]
        mask = self.to_host(idx, self._some_host(op)) if not idx.is_host else idx
        m = self._plain(mask)
        return self._shape_op(op, x, "Select", m, axis=op.attrs["axis"])

    def _some_host(self, op):
        plc = op.placement
        return plc.owner if isinstance(plc, HostPlacement) else plc.owners[0]

    def op_Concat(self, op, ins):
        xs = [self.at(op, v) for v in ins]
        axis = op.attrs["axis"]
        x0 = xs[0]
        if x0.is_host:
            return LV(x0.plc, "tensor", x0.dtype,
                      self.sess.h("Concat", x0.host, *[x.v for x in xs], axis=axis))
        if all(isinstance(x.v, MV) for x in xs):
            r = self.sess.h("Concat", x0.plc.owners[0], *[HV(x0.plc.owners[0], x.v.v) for x in xs],
                            axis=axis)
            return LV(x0.plc, "tensor", x0.dtype, MV(x0.plc, r.v))
        xs = [x if not isinstance(x.v, MV) else self._share_public(x) for x in xs]
        return LV(x0.plc, "tensor", x0.dtype, fxp.concat(self.sess, [x.v for x in xs], axis))

    def _share_public(self, x: LV) -> LV:
        d = x.dtype
        bits = d.ring_bits if d.is_fixed else 64
        t = rep.from_public(self.sess, x.plc, x.v.v, bits)
        if d.is_fixed:
            return LV(x.plc, "tensor", d, RepFixed(t, d.fractional_precision, d.integral_precision))
        return LV(x.plc, "tensor", d, t)

    def op_Shape(self, op, ins):
        x = ins[0]
        plc = op.placement
        if isinstance(plc, HostPlacement):
            x = self.to_host(x, plc.owner) if x.is_host else x
            if x.is_host:
                return LV(plc, "shape", None, self.sess.h("Shape", plc.owner, x.v))
        if x.is_host:  # shapes are public: the owner's view of its tensor's shape
            return LV(plc, "shape", None, self.sess.h("Shape", x.host, x.v))
        return LV(plc, "shape", None, fxp.shape_of(self.sess, x.v))

    def _fill(self, op, ins, value):
        shape = tuple(self._plain(ins[0]))
        d = self._ret_dtype(op)
        plc = op.placement
        host = self._some_host(op)
        if d.is_fixed:
            v = R.fill(shape, value << d.fractional_precision, d.ring_bits, self.sess.device)
        else:
            v = torch.full(shape, value, dtype=torch_dtype_of(d), device=self.sess.device)
        if isinstance(plc, HostPlacement):
            return LV(plc, "tensor", d, HV(host, v))
        return LV(plc, "tensor", d, MV(plc, v))

    def op_Ones(self, op, ins):
        return self._fill(op, ins, 1)

    def op_Zeros(self, op, ins):
        return self._fill(op, ins, 0)

    def op_Decrypt(self, op, ins):
        from moose_amd.protocols import aes

        key, ct = ins
        return aes.decrypt_logical(self, op, key, ct)
