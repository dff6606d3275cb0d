"""Whole-evaluation hipGraphs for the stacked (single-GPU) runtime.

An evaluation of a computation on a :class:`StackedSession` is a long, fixed sequence of
small kernels (a fixed-point sigmoid alone is ~100 launches), so at moderate tensor sizes
it is bound by Python dispatch and launch latency, not by the GPU.  For a given
(computation, argument signature) this module records the evaluation once into a HIP
graph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and afterwards replays it:

1. **warm-up run** (eager): produces the first result, sizes every workspace, and records
   each host->device upload made during the run (public constants; see
   ``ring.to_device``);
2. **capture run**: the same evaluation on a fresh session whose PRF keys live in a
   *frozen* :class:`~moose_amd.runtime.keys.KeyTable` (the kernels read keys from device
   memory, never from launch parameters), arguments in static device buffers, and every
   upload served from a copy staged before the capture (checked against the warm-up's
   bytes: a data-dependent upload aborts the capture);
3. **replay**: copy the new arguments into the static buffers, refresh the key table
   with fresh random keys (so each replay draws independent randomness -- the nonce
   sequence is fixed, the keys are not), replay, decode the outputs.

Host ``Load`` / ``Save`` are served at the replay's edges by a
:class:`~moose_amd.runtime.storage_tap.StorageTap` (loaded values are static buffers
refreshed from the storage before each replay, saved values are read back after it); the
plan is specialised on the stored values' shapes and dtypes as on the arguments'.  Anything
else that cannot be captured (share checkpoints, data-dependent uploads, CPU devices) falls
back to eager evaluation.
"""
from __future__ import annotations

import os
import warnings
from typing import Dict

import numpy as np
import torch

from moose_amd import errors
from moose_amd.ops import ring as R
from moose_amd.runtime.interpreter import Interpreter
from moose_amd.runtime.interpreter import dtype_of_numpy
from moose_amd.runtime.interpreter import numpy_to_torch
from moose_amd.runtime.keys import KeyTable
from moose_amd.runtime.session import StackedSession

SEGMENT_OPS = int(os.environ.get("MOOSEX_GRAPH_SEGMENT_OPS", "32"))


class CaptureError(errors.Unexpected):
    pass


class _Recorder:
    def __init__(self):
        self.items = []  # (host copy, device tensor)

    def __call__(self, t, device):
        d = t.to(device)
        self.items.append((t.detach().clone(), d))
        return d


class _Stager:
    def __init__(self, recorded, device):
        self.host = [h for h, _ in recorded]
        self.dev = [h.to(device) for h in self.host]  # staged before the capture begins
        self.i = 0

    def __call__(self, t, device):
        # Uploads come in warm-up order; some warm-up uploads are served from constant
        # caches during the capture (ring.fill / ring.weighted_sum), so skip forward to
        # the next recorded upload with the same bytes.
        tc = t.cpu()
        for i in range(self.i, len(self.host)):
            h = self.host[i]
            if h.dtype == tc.dtype and h.shape == tc.shape and torch.equal(h, tc):
                self.i = i + 1
                return self.dev[i]
        raise CaptureError("data-dependent host->device upload")


def _upload_hook(hook):
    class _Ctx:
        def __enter__(self):
            self.prev = R.set_upload_hook(hook)

        def __exit__(self, *exc):
            R.set_upload_hook(self.prev)

    return _Ctx()


def signature(arguments: dict):
    """Hashable description of the arguments a plan is specialised on."""
    sig = []
    for k in sorted(arguments):
        v = arguments[k]
        if isinstance(v, (np.ndarray, np.generic)) or (
                isinstance(v, (list, tuple)) and v and not isinstance(v[0], (str, bytes))):
            a = np.asarray(v)
            sig.append((k, "array", a.shape, a.dtype.str))
        elif isinstance(v, torch.Tensor):
            sig.append((k, "tensor", tuple(v.shape), str(v.dtype)))
        else:
            sig.append((k, "value", repr(v)))
    return tuple(sig)


def capturable(comp) -> bool:
    """Can an evaluation of ``comp`` be replayed?  Host Load / Save go through a StorageTap;
    share checkpoints and computed keys keep the computation eager."""
    from moose_amd.runtime import storage_tap

    return storage_tap.capturable(comp)


def storage_signature(comp, storage, hosts=None, arguments=None):
    """What ``comp``'s Loads read (runtime/storage_tap.signature): part of a plan's key."""
    from moose_amd.runtime import storage_tap

    if not any(op.kind == "Load" for op in comp.operations):
        return ()
    return storage_tap.signature(comp, storage, hosts, arguments)


class GraphPlan:
    """One captured evaluation (see module docstring)."""

    def __init__(self, comp, arguments: dict, device, storage, fixedpoint_ring, seed=None,
                 lanes=None):
        self.comp = comp
        self.device = torch.device(device)
        self.seed = seed
        self.ring = fixedpoint_ring
        self.storage = storage
        self.static = {}
        for k, v in arguments.items():
            if isinstance(v, (np.ndarray, np.generic)) or (
                    isinstance(v, (list, tuple)) and v and not isinstance(v[0], (str, bytes))):
                a = np.asarray(v)
                t = numpy_to_torch(a, self.device)
                t._moose_dtype = dtype_of_numpy(a)
                self.static[k] = t
            else:
                self.static[k] = v
        # 1. warm-up (eager): first result + recorded uploads.  It runs on the stream (and
        # the dataflow lanes) the capture will use, so per-stream GEMM workspaces are sized
        # before the capture (no allocation while capturing)
        stream = torch.cuda.Stream(self.device)
        rec = _Recorder()
        sess = StackedSession(self.device, seed=seed)
        interp = Interpreter(sess, storage, fixedpoint_ring, lanes=lanes)
        with _upload_hook(rec), torch.cuda.stream(stream):
            outs = interp.run(comp, self.static)
            self.first = self._decode(interp, outs)
        self.stats = sess.stats
        torch.cuda.synchronize(self.device)
        # host Load / Save at the replay's edges (static buffers staged before the capture)
        from moose_amd.runtime.storage_tap import StorageTap

        self.tap = StorageTap(comp, storage, self.device, arguments=arguments)
        # 2. capture on a session with a frozen, refreshed key table
        self.keys = KeyTable(self.device, capacity=max(256, sess.keytable.n + 16))
        self.keys.refresh()
        self.keys.frozen = True
        self.sess = StackedSession(self.device, seed=seed)
        self.sess.use_keytable(self.keys)
        self.interp = Interpreter(self.sess, storage, fixedpoint_ring, lanes=lanes)
        self.interp.lanes = interp.lanes  # the warm-up's streams
        stager = _Stager(rec.items, self.device)
        torch.cuda.synchronize(self.device)
        # The evaluation is captured as a chain of graphs of SEGMENT_OPS logical ops each
        # (sharing one memory pool, replayed in capture order): a single graph of 10^5+
        # kernel nodes is slow to instantiate and has crashed the HIP runtime.
        self.graphs = []
        pool = torch.cuda.graph_pool_handle()
        state = {"g": None, "n": 0}

        lanes = self.interp.lanes

        def begin():
            g = torch.cuda.CUDAGraph()
            # thread-local: only this thread's calls can invalidate the capture -- a
            # process-group watchdog thread polling its events (multi-rank runs) cannot
            g.capture_begin(pool=pool, capture_error_mode="thread_local")
            state["g"], state["n"] = g, 0
            if lanes is not None:  # the lanes join this segment's capture
                lanes.fork()

        def end():
            if lanes is not None:  # ... and are joined back before it ends
                lanes.join()
            state["g"].capture_end()
            self.graphs.append(state["g"])

        def rotate():  # called before each op: segments never end empty-handed
            if state["g"] is None:
                begin()
            elif state["n"] >= SEGMENT_OPS:
                end()
                begin()
            state["n"] += 1

        self.interp.on_op = rotate
        self.interp.storage_tap = self.tap
        with _upload_hook(stager), torch.cuda.stream(stream):
            try:
                self.outs = self.interp.run(comp, self.static)
            except BaseException:
                if os.environ.get("MOOSEX_GRAPHS_DEBUG") == "1":
                    import sys
                    import traceback

                    traceback.print_exc(file=sys.stderr)
                    sys.stderr.flush()
                raise
            finally:
                if state["g"] is not None:
                    end()
        self.interp.on_op = None
        self.interp.storage_tap = None
        torch.cuda.synchronize(self.device)
        self._stager = stager  # keep the staged constants alive
        self.replays = 0
        self.t_graph, self.t_eager = [], []
        self._warm = False
        self.decision = "graph" if PROBES <= 0 else None

    def next_mode(self) -> str:
        """"graph" / "eager" once decided; while measuring, "probe" (a timed replay) and
        "eager" (a timed eager evaluation) alternate, after one untimed replay (a graph's
        first launch uploads it)."""
        if self.decision is not None:
            return self.decision
        if not self._warm:
            self._warm = True
            return "graph"
        if len(self.t_graph) < PROBES or len(self.t_eager) < PROBES:
            return "probe" if len(self.t_graph) <= len(self.t_eager) else "eager"
        med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
        self.decision = "graph" if med(self.t_graph) <= med(self.t_eager) else "eager"
        return self.decision

    def _decode(self, interp, outs) -> Dict[str, np.ndarray]:
        res = {}
        for tag, lv in outs.items():
            if lv.kind == "unit":
                continue
            res[tag] = interp.to_numpy(lv)
        return res

    def run(self, arguments: dict) -> Dict[str, np.ndarray]:
        for k, v in arguments.items():
            t = self.static.get(k)
            if isinstance(t, torch.Tensor):
                a = np.asarray(v)
                a = a.view(np.int64) if a.dtype == np.uint64 else a
                # a pageable copy straight from the caller's array, as the eager path does:
                # HIP's staged DMA (0.155 ms for 8 MB on MI355X) beats a host memcpy into a
                # pinned buffer followed by a blit (0.321 ms; profiles/r3_graphs_vs_eager.md)
                src = torch.from_numpy(np.ascontiguousarray(a).reshape(t.shape))
                t.copy_(src if src.dtype == t.dtype else src.to(t.dtype))
        self.tap.refresh(self.storage)  # the stored values this replay loads
        if self.seed is None:
            self.keys.refresh(self.keys.n)  # fresh randomness for this replay (used slots)
        else:  # a seeded evaluation: the seeded session's keys, as the eager run draws them
            self.keys.refresh_seeded(self.seed)
        for g in self.graphs:
            g.replay()
        self.replays += 1
        self.tap.write_saves(self.storage)  # what it saved, read back into the storage
        return self._decode(self.interp, self.outs)


PROBES = int(os.environ.get("MOOSEX_GRAPHS_PROBES", "0"))


class GraphCache:
    """Per-runtime cache of captured plans keyed by (computation, argument signature).

    Replay is the default on every shape (``MOOSEX_GRAPHS_PROBES=0``): with arguments
    uploaded the way the eager path uploads them, a replay is never slower than the eager
    evaluation on the reference dot sweep (profiles/r3_graphs_vs_eager.md).  Adaptive mode
    (``MOOSEX_GRAPHS_PROBES=k > 0``): after the capture a plan times ``k`` replays and ``k``
    eager evaluations, alternating (the caller runs the eager ones and reports them through
    :meth:`note_eager`), and keeps the faster mode by median -- a guard for programs whose
    device work dwarfs dispatch, at the price of decisions made on a few noisy samples."""

    def __init__(self):
        self.plans = {}
        self.failed = set()
        self._eager_key = None

    def evaluate(self, comp, arguments, device, storage, ring, seed=None, lanes=None):
        if not capturable(comp):
            return None
        key = (id(comp), signature(arguments),
               storage_signature(comp, storage, arguments=arguments))
        self._eager_key = None
        plan = self.plans.get(key)
        if plan is not None and plan.comp is comp:
            mode = plan.next_mode()
            if mode == "eager":
                self._eager_key = key  # the caller evaluates eagerly and reports the time
                return None
            import time

            t0 = time.perf_counter()
            res = plan.run(arguments)
            if mode == "probe":
                plan.t_graph.append(time.perf_counter() - t0)
            return res, plan.stats
        if key in self.failed or not capturable(comp):
            return None
        try:
            plan = GraphPlan(comp, arguments, device, storage, ring, seed, lanes=lanes)
        except Exception as e:  # noqa: BLE001 - any capture failure means "run eagerly"
            import traceback

            self.last_error = traceback.format_exc()
            if os.environ.get("MOOSEX_GRAPHS_DEBUG") == "1":
                raise
            warnings.warn(f"hipGraph capture failed, evaluating eagerly: {e}")
            self.failed.add(key)
            try:
                torch.cuda.synchronize()
            except Exception:  # noqa: BLE001
                pass
            return None
        self.plans[key] = plan
        return plan.first, plan.stats

    def note_eager(self, seconds: float):
        """Time of the eager evaluation that evaluate() just handed to the caller."""
        key, self._eager_key = self._eager_key, None
        plan = self.plans.get(key) if key is not None else None
        if plan is not None and plan.decision is None:
            plan.t_eager.append(seconds)
