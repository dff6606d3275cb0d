"""Replayed one-party-per-GPU evaluations: the SPMD tape.

An SPMD evaluation (``parallel/spmd.py``: one process per party, every reshare a
point-to-point message) of a latency-bound program -- the tutorial LR inference is 73
message rounds of a few small kernels each -- costs per-op Python dispatch in every
process on top of the message latency.  The reference pre-wires every operation as a
task of a compiled host graph once per session (``execution/asynchronous.rs:456-530``);
here an evaluation is recorded once and replayed:

1. **warm-up** (eager, message plans recording): the first result; sizes every
   workspace; records the host->device uploads (public constants) and, through the
   transport's message plan, the header of every message;
2. **capture** on a fresh session over a *frozen* key table: the interpreter runs the
   program again with its kernels captured as hipGraph segments (``torch.cuda.CUDAGraph``
   is hipGraph on ROCm) and the transport in tape mode, so every message round ends the
   current segment and is recorded as a :class:`~moose_amd.parallel.transport.CommStep`
   (its device buffers, peers and order) instead of being sent;
3. **replay**: copy the new arguments into the static buffers, refresh the key table
   (fresh keys per evaluation; the key exchange of the setup is one of the taped rounds),
   then walk the tape -- replay a segment, issue a round (one grouped exchange, no header,
   no Python op dispatch), replay the next segment ... -- and decode the outputs.

Every process runs the same program, so every process's tape has the same rounds in the
same order and replays pair up exactly as the eager evaluations did.  Whether to tape is
decided collectively (an all-reduce of every rank's capture outcome): a program that one
process cannot capture runs eagerly everywhere.

Deterministic (seeded) sessions replay bitwise like a fresh eager seeded session: the
replay re-draws the seeded keys in the order the eager setup would.
"""
from __future__ import annotations

import os
import time
import warnings
from typing import Dict
from typing import Optional

import numpy as np
import torch

from moose_amd.ops import native as nat
from moose_amd.parallel.transport import CommStep
from moose_amd.runtime import graphs as G
from moose_amd.runtime.interpreter import Interpreter
from moose_amd.runtime.interpreter import dtype_of_numpy
from moose_amd.runtime.interpreter import numpy_to_torch
from moose_amd.runtime.keys import KeyTable

SEGMENT_OPS = G.SEGMENT_OPS


class SPMDTape:
    """One recorded SPMD evaluation of this process (module doc)."""

    def __init__(self, comp, arguments: dict, identity: str, role_ranks: Dict[str, int],
                 tr, device, storage, ring: int, seed: Optional[int] = None, warm=None,
                 keep_graph: bool = False, shared_static: Optional[dict] = None):
        """``warm``: the warm-up already ran elsewhere (the in-process parties of
        parallel/threads.py run it together, on threads) -- a dict with the recorded
        ``uploads``, the ``first`` outputs, the session ``stats`` and the number of key
        slots ``keys_n`` it used.  ``keep_graph``: the segments keep their hipGraph (not
        instantiated until a replay) so a caller can compose them into a larger graph.
        ``shared_static``: argument buffers shared by the tapes of one device (the graphs
        only read them), so a replay uploads each argument once per device."""
        from moose_amd.parallel.spmd import SPMDSession

        self.comp, self.device, self.tr = comp, torch.device(device), tr
        self.identity, self.role_ranks, self.seed = identity, dict(role_ranks), seed
        self.static = {}
        self.owns_static = set()  # the buffers this tape uploads (the others' are shared)
        for k, v in arguments.items():
            if isinstance(v, (np.ndarray, np.generic)) or (
                    isinstance(v, (list, tuple)) and v and not isinstance(v[0], (str, bytes))):
                a = np.asarray(v)
                t = shared_static.get(k) if shared_static is not None else None
                if t is None or tuple(t.shape) != a.shape or \
                        getattr(t, "_moose_dtype", None) != dtype_of_numpy(a):
                    t = numpy_to_torch(a, self.device)
                    t._moose_dtype = dtype_of_numpy(a)
                    self.owns_static.add(k)
                    if shared_static is not None:
                        shared_static[k] = t
                self.static[k] = t
            else:
                self.static[k] = v
        stream = torch.cuda.Stream(self.device)
        if warm is None:
            # 1. warm-up: the first result, the message plan, the uploads
            rec = G._Recorder()
            sess = SPMDSession(identity, role_ranks, tr, device=self.device, seed=seed)
            interp = Interpreter(sess, storage, ring)
            with G._upload_hook(rec), torch.cuda.stream(stream):
                outs = interp.run(comp, self.static)
                self.first = self._decode(interp, sess, outs)
            self.stats = sess.stats
            uploads, keys_n = rec.items, sess.keytable.n
        else:
            uploads, keys_n = warm["uploads"], warm["keys_n"]
            self.first, self.stats = warm["first"], warm["stats"]
        torch.cuda.synchronize(self.device)
        # 2. capture: frozen keys, transport in tape mode
        self.keys = KeyTable(self.device, capacity=max(64, keys_n + 16))
        self.keys.frozen = True
        self.sess = SPMDSession(identity, role_ranks, tr, device=self.device, seed=seed)
        self.sess.use_keytable(self.keys)
        self.sess.key_setups = []
        self.interp = Interpreter(self.sess, storage, ring)
        # this party's host Load / Save at the replay's edges (runtime/storage_tap.py)
        from moose_amd.runtime.storage_tap import StorageTap

        self.storage = storage
        self.tap = StorageTap(comp, storage, self.device, hosts={identity},
                              arguments=arguments)
        self.interp.storage_tap = self.tap
        stager = G._Stager(uploads, self.device)
        self.steps = []  # CUDAGraph segments and CommSteps, in program order
        pool = torch.cuda.graph_pool_handle()
        state = {"g": None, "n": 0}

        def begin():
            g = torch.cuda.CUDAGraph(keep_graph=keep_graph)
            g.capture_begin(pool=pool, capture_error_mode="thread_local")
            state["g"], state["n"] = g, 0

        def end():
            g = state["g"]
            if g is not None:
                state["g"] = None  # ended once, also when the capture failed
                with warnings.catch_warnings():  # a segment between two rounds may be empty
                    warnings.filterwarnings("ignore", message="The CUDA Graph is empty")
                    g.capture_end()
                if state["n"]:
                    self.steps.append(g)

        def rotate():  # before each op: bounded segments
            if state["g"] is None:
                begin()
            elif state["n"] >= SEGMENT_OPS:
                end()
                begin()
            state["n"] += 1

        def on_comm(step: CommStep):
            state["n"] += 1  # the segment holds the round's send copies, if any
            end()
            self.steps.append(step)
            begin()

        torch.cuda.synchronize(self.device)
        self.interp.on_op = rotate
        tr.tape = on_comm
        try:
            with G._upload_hook(stager), torch.cuda.stream(stream):
                try:
                    begin()
                    self.outs = self.interp.run(comp, self.static)
                finally:
                    end()
        finally:
            tr.tape = None
            self.interp.on_op = None
            self.interp.storage_tap = None
        torch.cuda.synchronize(self.device)
        self._stager = stager  # the staged constants stay alive with the graphs
        self.stream = stream
        self.rounds = sum(isinstance(s, CommStep) for s in self.steps)
        self.segments = len(self.steps) - self.rounds
        self.replays = 0
        self.issue_s = []  # host time per replay spent issuing (graphs + message calls)
        self.comm_host_s = []  # host time per replay inside the message rounds
        # per replay, with MOOSEX_TAPE_TIMING=1: the tape stream's time inside the message
        # rounds (events around each round: transfer + waiting for the peers), summed and
        # the longest round -- p50 ~ rounds x round latency + kernel time, from the record
        self.timing = os.environ.get("MOOSEX_TAPE_TIMING") == "1"
        self.round_device_ms, self.round_device_max_ms = [], []
        if seed is None:  # unseeded replays draw their keys on the device (keys.py)
            self.keys.enable_device_refresh()
        self._pinned = {}  # argument name -> pinned host staging buffer

    # ------------------------------------------------------------------------------
    def _decode(self, interp, sess, outs) -> Dict[str, np.ndarray]:
        if interp is getattr(self, "interp", None) and self.tap.save_keys:
            self.tap.write_saves(self.storage)  # a replay's saved values, into the storage
        res = {}
        for tag, lv in outs.items():
            if lv.kind == "unit" or not sess.materialized(lv.v):
                continue
            res[tag] = interp.to_numpy(lv)
        return res

    def _fill_keys(self):
        """Fresh keys for this replay.  Unseeded: random slots; the taped setup rounds
        overwrite the peers' slots with their keys.  Seeded: the draws a fresh seeded
        session makes in its setups (SPMDSession.setup), in the same order."""
        if self.seed is None:
            self.keys.refresh_device(self.keys.n)
            return
        rng = torch.Generator().manual_seed(self.seed)
        draw = lambda: bytes(torch.randint(0, 256, (16,), generator=rng,  # noqa: E731
                                           dtype=torch.uint8).tolist())
        for base, idx in self.sess.key_setups:
            if base == "seed":  # a fresh seed (SPMDSession.h_fresh_seed): one draw
                b = draw()
                if idx is not None:
                    self.keys._write(idx, [b])
                continue
            allk = [draw() for _ in range(4)]
            if idx is None:
                continue
            for _ in range(4):  # the member's alloc(4) draws too (SPMDSession.setup)
                draw()
            allk[(idx + 2) % 3] = bytes(16)
            self.keys._write(base, allk)

    def pinned(self, k):
        """(pinned host tensor, its numpy view): the staging buffer of argument ``k``."""
        t = self.static[k]
        pin = self._pinned.get(k)
        if pin is None or pin[0].shape != t.shape or pin[0].dtype != t.dtype:
            pt = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            pin = self._pinned[k] = (pt, pt.numpy())
        return pin

    def uploads(self):
        """[(device buffer, pinned staging buffer)] of the arguments this tape uploads (a
        composed graph copies them itself: PartyTapes._compose)."""
        return [(self.static[k], self.pinned(k)[0]) for k in sorted(self.owns_static)
                if isinstance(self.static.get(k), torch.Tensor) and self.static[k].is_cuda]

    def copy_arguments(self, arguments: dict, upload: bool = True):
        """The new arguments into the static buffers, on the current stream: through a
        pinned staging buffer per argument (an asynchronous DMA; a pageable copy would hold
        the host until it ran).  The previous replay has completed (its outputs were
        decoded), so the staging buffer is free.  ``upload=False``: only staged (the graph
        holds the copies)."""
        for k, v in arguments.items():
            t = self.static.get(k)
            if not isinstance(t, torch.Tensor) or k not in self.owns_static:
                continue
            a = np.asarray(v)
            a = a.view(np.int64) if a.dtype == np.uint64 else a
            if t.device.type != "cuda":
                src = torch.from_numpy(np.ascontiguousarray(a).reshape(t.shape))
                t.copy_(src if src.dtype == t.dtype else src.to(t.dtype))
                continue
            pin = self.pinned(k)
            np.copyto(pin[1], a.reshape(t.shape), casting="unsafe")  # no torch dispatch
            if upload:
                nat.check(nat.lib().mx_copy_async(t.data_ptr(), pin[0].data_ptr(),
                    t.numel() * t.element_size(),
                    torch.cuda.current_stream(t.device).cuda_stream), "argument upload")
        if self.tap.loads:  # the stored values this replay loads, as arguments
            self.tap.refresh(self.storage)

    def replay(self, arguments: dict) -> Dict[str, np.ndarray]:
        with torch.cuda.stream(self.stream):
            self.copy_arguments(arguments)
            self._fill_keys()
            issue = 0.0
            tr = self.tr
            staged = tr.stage
            timing = self.timing and self.device.type == "cuda"
            evs = []
            comm_host = 0.0
            for s in self.steps:
                t0 = time.perf_counter()
                if isinstance(s, CommStep):
                    if timing:
                        e0 = torch.cuda.Event(enable_timing=True)
                        e0.record(self.stream)
                    s.run(tr)
                    if timing:
                        e1 = torch.cuda.Event(enable_timing=True)
                        e1.record(self.stream)
                        evs.append((e0, e1))
                    dt = time.perf_counter() - t0
                    comm_host += dt
                    if not staged:  # a staged (gloo) round's time is host copies, not issue
                        issue += dt
                else:
                    s.replay()
                    issue += time.perf_counter() - t0
            self.issue_s.append(issue)
            self.comm_host_s.append(comm_host)
            self.replays += 1
            out = self._decode(self.interp, self.sess, self.outs)
            if timing:  # the decode synchronised the tape stream: the events are complete
                ms = [a.elapsed_time(b) for a, b in evs]
                self.round_device_ms.append(sum(ms))
                self.round_device_max_ms.append(max(ms) if ms else 0.0)
            # every send-only round of this replay confirmed ON THE TAPE STREAM: under RCCL
            # a send's completion wait is a stream dependency, so the next replay's
            # kernels -- which rewrite the static buffers those sends read -- are ordered
            # after them by the tape itself, not by a caller's device-wide synchronize
            end = getattr(tr, "end_evaluation", None)
            if end is not None:
                end()
        return out


# ------------------------------------------------------------------------------------------
# per-process cache with a collective decision
# ------------------------------------------------------------------------------------------
_TAPES: Dict[tuple, object] = {}
_SEEN: Dict[tuple, int] = {}
MAX_TAPES = 32


def enabled(device) -> bool:
    return torch.device(device).type == "cuda" and os.environ.get("MOOSEX_SPMD_GRAPHS",
                                                                   "1") != "0"


def _agree(tr, ok: bool) -> bool:
    """Every rank of the transport's group learns whether all of them succeeded.  The
    transport's group must be exactly the session's ranks (a transport on the default group
    of a larger job would wait for ranks that are not in this evaluation)."""
    import torch.distributed as dist

    if tr.world <= 1:
        return ok
    nccl = dist.get_backend(tr.group) == "nccl"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                     device=tr.device if nccl else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=tr.group)
    return bool(t.item())


def storage_key(comp, storage, identity: str, tr, arguments=None) -> Optional[int]:
    """A key of what ``comp``'s Loads read from storage, the SAME on every rank: each rank
    hashes the (key, shape, dtype) of the values its own identity loads
    (runtime/storage_tap.signature) and the group sums the hashes.  A stored value only its
    owner can see is then part of every rank's message-plan and tape key, so a changed shape
    re-records the plan everywhere instead of desynchronising the replay.  None when
    ``comp`` loads nothing or cannot be taped (the headers are sent)."""
    import hashlib

    import torch.distributed as dist

    if not any(op.kind == "Load" for op in comp.operations) or not G.capturable(comp):
        return None
    sig = G.storage_signature(comp, storage, hosts={identity}, arguments=arguments)
    h = int.from_bytes(hashlib.blake2b(repr(sig).encode(), digest_size=7).digest(), "little")
    if tr.world <= 1:
        return h
    nccl = dist.get_backend(tr.group) == "nccl"
    t = torch.tensor([h], dtype=torch.int64, device=tr.device if nccl else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=tr.group)
    return int(t.item())


def evaluate(comp, arguments: dict, identity: str, role_ranks: Dict[str, int], tr, device,
             storage, ring: int, seed: Optional[int] = None):
    """Evaluate ``comp`` as ``identity`` through the tape cache: the first evaluation of a
    (program, argument signature) runs eagerly, the second is captured (every rank, then a
    collective decision) and replayed, later ones replay.  Returns ``(outputs, stats,
    tape-or-None)``; None when the caller must run eagerly (first sight, not capturable,
    or a failed capture on any rank)."""
    from moose_amd.parallel.spmd import _argument_key
    from moose_amd.parallel.spmd import _loads
    from moose_amd.parallel.spmd import _structure_key

    skey = getattr(tr, "storage_key", None)  # the caller's collective storage_key()
    if not enabled(device) or not getattr(tr, "plans", False) \
            or (_loads(comp) and skey is None) or not G.capturable(comp):
        return None
    key = (tr.plan_scope, tr.rank, tr.world, id(tr.group), identity,
           tuple(sorted(role_ranks.items())), _structure_key(comp), _argument_key(arguments),
           G.signature(arguments), seed, skey)
    tape = _TAPES.get(key)
    if tape is not None:
        if tape is False:
            return None
        return tape.replay(arguments), tape.stats, tape
    n = _SEEN.get(key, 0) + 1
    _SEEN[key] = n
    if n < 2:  # the eager evaluation records the message plan first
        return None
    tape, err = None, None
    try:
        tape = SPMDTape(comp, arguments, identity, role_ranks, tr, device, storage, ring, seed)
    except Exception as e:  # noqa: BLE001 - any capture failure: eager, on every rank
        err = e
        try:
            torch.cuda.synchronize(device)
        except Exception:  # noqa: BLE001
            pass
    if not _agree(tr, tape is not None):
        if os.environ.get("MOOSEX_GRAPHS_DEBUG") == "1" and err is not None:
            raise err
        _TAPES[key] = False
        return None
    if len(_TAPES) >= MAX_TAPES:
        _TAPES.pop(next(iter(_TAPES)))
    _TAPES[key] = tape
    return tape.first, tape.stats, tape
