"""``LocalMooseRuntime``: all identities simulated in one process on one device -- or,
with ``device_map={identity: device}``, every identity a thread of this process on its
own GPU, exchanging device-to-device copies (parallel/threads.py).

With ``use_graphs=True`` (or ``MOOSEX_GRAPHS=1``) repeated evaluations of the same
computation and argument signature replay a captured hipGraph (runtime/graphs.py).

Parity: reference ``pymoose/pymoose/runtime.py:14-70`` + ``pymoose/src/bindings.rs:137-250``
(``AsyncTestRuntime``, ``execution/asynchronous.rs:634-773``).  Here the three parties of
each replicated placement are stacked on one device (an MI355X when available, else the
CPU), so every protocol step is one kernel launch for all parties.
"""
from __future__ import annotations

import os
import time
import weakref
from typing import Dict
from typing import List
from typing import Optional

import numpy as np
import torch

from moose_amd.computation import computation as ecomp
from moose_amd.ir.computation import Computation
from moose_amd.runtime.interpreter import Interpreter
from moose_amd.runtime.session import StackedSession


def default_device():
    dev = os.environ.get("MOOSEX_DEVICE")
    if dev:
        return dev
    return "cuda" if torch.cuda.is_available() else "cpu"


def to_native(computation, fixedpoint_ring=128) -> Computation:
    """Accept an AbstractComputation, an eDSL Computation, a native Computation, a
    MooseComputation, or serialized bytes; return a native-IR Computation."""
    from moose_amd.compiler.from_edsl import convert
    from moose_amd.edsl import base as edsl
    from moose_amd.edsl import tracer

    if isinstance(computation, Computation):
        return computation
    if hasattr(computation, "native"):  # MooseComputation
        return computation.native
    if isinstance(computation, edsl.AbstractComputation):
        computation = tracer.trace(computation)
    if isinstance(computation, (bytes, bytearray)):
        from moose_amd.computation import utils

        try:
            return Computation.from_msgpack(bytes(computation))
        except Exception:
            computation = utils.deserialize_computation(bytes(computation))
    if isinstance(computation, ecomp.Computation):
        return convert(computation, fixedpoint_ring)
    raise ValueError(f"cannot evaluate object of type {type(computation)}")


class LocalMooseRuntime:
    """Locally simulated runtime with optional per-identity storage."""

    def __init__(
        self,
        identities: List[str],
        storage_mapping: Optional[Dict[str, Dict]] = None,
        device=None,
        fixedpoint_ring: int = 128,
        seed: Optional[int] = None,
        use_graphs: Optional[bool] = None,
        lanes: Optional[int] = None,
        device_map: Optional[Dict[str, str]] = None,
        timeout: Optional[float] = None,
    ):
        identities = [getattr(i, "name", i) for i in identities]
        storage_mapping = dict(storage_mapping or {})
        for ident in storage_mapping:
            if ident not in identities:
                raise ValueError(
                    f"Found unknown identity {ident} in `storage_mapping` arg, "
                    f"must be one of {identities}."
                )
        self.identities = identities
        self.storage = {i: dict(storage_mapping.get(i, {})) for i in identities}
        self.device = torch.device(device or default_device())
        self.fixedpoint_ring = fixedpoint_ring
        self.seed = seed
        self.last_stats = None
        self.last_replay = None  # parties on GPUs: how the last replay ran (PartyTapes)
        self.last_timings = None
        # replay whole evaluations as hipGraphs (runtime/graphs.py).  Default (None): on a
        # GPU, "auto" -- a computation evaluated a second time with the same argument
        # signature, whose eager evaluation was dispatch-bound (under AUTO_GRAPH_MS), is
        # captured then and replayed from the third evaluation on; True captures at the
        # first evaluation; False (or MOOSEX_GRAPHS=0) never captures.
        if use_graphs is None:
            env = os.environ.get("MOOSEX_GRAPHS", "auto")
            use_graphs = {"1": True, "0": False}.get(env, "auto")
        self.use_graphs = use_graphs
        # auto mode: (id(comp), signature) -> (weak reference to comp, last eager seconds);
        # weak, so the cache does not keep the user's computations alive
        self._seen = {}
        # HIP streams for independent operations (runtime/lanes.py); MOOSEX_LANES=n
        self.lanes = lanes
        from moose_amd.runtime.graphs import GraphCache

        self._graphs = GraphCache()
        self._native_cache = {}
        # parties as threads, each on its own device (parallel/threads.py): {identity:
        # device}; identities not named run on ``device``
        self.device_map = None
        if device_map:
            unknown = set(device_map) - set(identities)
            if unknown:
                raise ValueError(f"`device_map` names unknown identities {sorted(unknown)}")
            self.device_map = {i: torch.device(device_map.get(i, self.device))
                               for i in identities}
        self.timeout = timeout
        self.last_stats_by_identity = None
        self._party_tapes = {}  # (id(comp), signature) -> (comp, PartyTapes or False)

    def set_default(self):
        from moose_amd.edsl.base import set_current_runtime

        set_current_runtime(self)

    # ------------------------------------------------------------------
    def _native(self, computation) -> Computation:
        """to_native, memoised per traced object: re-evaluating the same
        AbstractComputation skips tracing + conversion and keeps the Computation's
        identity stable, so captured hipGraph plans are found again."""
        if isinstance(computation, Computation):
            return computation
        hit = self._native_cache.get(id(computation))
        if hit is not None and hit[0] is computation:
            return hit[1]
        comp = to_native(computation, self.fixedpoint_ring)
        if len(self._native_cache) >= 64:
            self._native_cache.pop(next(iter(self._native_cache)))
        self._native_cache[id(computation)] = (computation, comp)
        return comp

    def evaluate_computation(self, computation, arguments=None, compiler_passes=None):
        comp = self._native(computation)
        if compiler_passes:
            from moose_amd.compiler import passes

            comp = passes.compile(comp, compiler_passes, arg_specs=arg_specs_of(arguments),
                                  fixedpoint_ring=self.fixedpoint_ring)
        return self.evaluate_compiled(comp, arguments)

    def evaluate_compiled(self, comp, arguments=None):
        comp = to_native(comp, self.fixedpoint_ring)
        arguments = dict(arguments or {})
        if self.device_map is not None:
            return self._evaluate_parties(comp, arguments)
        if _is_lowered(comp):
            from moose_amd.runtime.graph_executor import GraphExecutor

            ex = GraphExecutor(self.device, self.storage)
            t0 = time.perf_counter()
            outs = ex.run(comp, arguments)
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self.last_timings = {i: int((time.perf_counter() - t0) * 1e6) for i in self.identities}
            from moose_amd.runtime.distributed import _host_numpy

            return {k: _host_numpy(v) for k, v in outs.items()}
        graphs = self.use_graphs and self.device.type == "cuda"
        akey = None
        if graphs and self.use_graphs == "auto":
            from moose_amd.runtime.graphs import signature

            akey = (id(comp), signature(arguments))
            seen = self._seen.get(akey)
            graphs = (seen is not None and seen[0]() is comp and seen[1] < AUTO_GRAPH_MS / 1e3)
        if graphs:
            t0 = time.perf_counter()
            r = self._graphs.evaluate(comp, arguments, self.device, self.storage,
                                      self.fixedpoint_ring, self.seed, lanes=self.lanes)
            if r is not None:
                result, self.last_stats = r
                torch.cuda.synchronize(self.device)
                elapsed = int((time.perf_counter() - t0) * 1e6)
                self.last_timings = {i: elapsed for i in self.identities}
                return result
        sess = StackedSession(self.device, seed=self.seed)
        interp = Interpreter(sess, self.storage, self.fixedpoint_ring, lanes=self.lanes)
        t0 = time.perf_counter()
        outs = interp.run(comp, arguments)
        result = {}
        for tag, lv in outs.items():
            if lv.kind == "unit":
                continue
            result[tag] = interp.to_numpy(lv)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - t0
        if graphs:
            self._graphs.note_eager(dt)  # adaptive replay: the plan's eager probe
        if akey is not None:
            if len(self._seen) >= 256:
                self._seen.pop(next(iter(self._seen)))
            self._seen[akey] = (weakref.ref(comp), dt)
        elapsed = int(dt * 1e6)
        self.last_timings = {i: elapsed for i in self.identities}
        self.last_stats = sess.stats
        return result

    def _evaluate_parties(self, comp, arguments):
        """Parties as threads, one device each (parallel/threads.py).  On GPUs, a
        dispatch-bound evaluation seen a second time is recorded (per-party tapes) and
        replayed from then on by one host thread (PartyTapes), as the auto hipGraph mode
        of the stacked session."""
        from moose_amd.parallel import threads as T
        from moose_amd.runtime import graphs as G

        devices = [self.device_map[i] for i in self.identities]
        tapeable = (self.use_graphs and all(d.type == "cuda" for d in devices)
                    and os.environ.get("MOOSEX_SPMD_GRAPHS", "1") != "0"
                    and G.capturable(comp) and not _is_lowered(comp))
        key = None
        if tapeable:
            key = (id(comp), G.signature(arguments),
                   G.storage_signature(comp, self.storage, arguments=arguments))
            tapes = self._party_tapes.get(key)
            if tapes is not None and tapes[0] is comp and tapes[1] is not False:
                t0 = time.perf_counter()
                outs = tapes[1].replay(arguments)
                for d in set(devices):
                    torch.cuda.synchronize(d)
                elapsed = int((time.perf_counter() - t0) * 1e6)
                self.last_timings = {i: elapsed for i in self.identities}
                self.last_stats_by_identity = {i: t.stats for i, t in
                                               zip(self.identities, tapes[1].tapes)}
                self.last_stats = self.last_stats_by_identity[self.identities[0]]
                # how this replay ran (per-party graphs / composed / per-action) and whether
                # the per-party graphs passed their capture-time check
                self.last_replay = {"form": tapes[1].replay_form,
                                    "validated": tapes[1].validated,
                                    "fallback": tapes[1].fallback}
                result = {}
                for i in self.identities:
                    result.update(outs[i])
                return result
        seen = self._seen.get(key) if key is not None else None
        record = (tapeable and seen is not None and seen[0]() is comp
                  and (self.use_graphs is True or seen[1] < PARTIES_AUTO_GRAPH_MS / 1e3)
                  and key not in self._party_tapes)
        t0 = time.perf_counter()
        result, stats, self.last_timings, warm = T.run_parties(
            comp, arguments, self.identities, devices, self.storage, self.fixedpoint_ring,
            self.seed, timeout=self.timeout, record=record)
        dt = time.perf_counter() - t0
        self.last_stats_by_identity = stats
        self.last_stats = stats.get(self.identities[0])
        if key is not None:
            if len(self._seen) >= 256:
                self._seen.pop(next(iter(self._seen)))
            self._seen[key] = (weakref.ref(comp), dt)
        if record and warm is not None:
            try:
                tapes = T.PartyTapes(comp, arguments, self.identities, devices, self.storage,
                                     self.fixedpoint_ring, self.seed, warm)
            except Exception:  # noqa: BLE001 - not capturable: this signature stays eager
                if os.environ.get("MOOSEX_GRAPHS_DEBUG") == "1":
                    raise
                tapes = False
                for d in set(devices):
                    torch.cuda.synchronize(d)
            if len(self._party_tapes) >= 32:
                self._party_tapes.pop(next(iter(self._party_tapes)))
            self._party_tapes[key] = (comp, tapes)
        return result

    def read_value_from_storage(self, identity, key):
        if identity not in self.storage:
            raise RuntimeError(f"unknown identity {identity}")
        return self.storage[identity][key]

    def write_value_to_storage(self, identity, key, value):
        if identity not in self.storage:
            raise RuntimeError(f"unknown identity {identity}")
        self.storage[identity][key] = np.asarray(value) if not isinstance(value, str) else value


# auto hipGraph mode: only evaluations whose eager run took less than this are captured
# (dispatch-bound; a GEMM-bound evaluation gains nothing and its capture pins memory)
AUTO_GRAPH_MS = float(os.environ.get("MOOSEX_GRAPHS_AUTO_MS", "50"))
# the same for parties as threads: their eager evaluation is three Python dispatch loops
# sharing one interpreter lock, so a dispatch-bound program takes a few times longer
PARTIES_AUTO_GRAPH_MS = 4 * AUTO_GRAPH_MS


def _is_lowered(comp: Computation) -> bool:
    """A computation is host-level when every op is on a host placement and no op
    carries a logical (Tensor/Shape) type."""
    from moose_amd.compiler.passes import is_lowered

    return is_lowered(comp)


def arg_specs_of(arguments) -> dict:
    """Shapes of concrete arguments (lowering is shape-specialised)."""
    specs = {}
    for k, v in (arguments or {}).items():
        if isinstance(v, (str, bytes)):
            continue
        shape = tuple(v.shape) if hasattr(v, "shape") else tuple(np.shape(v))
        specs[k] = (shape, None)
    return specs
