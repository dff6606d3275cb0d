"""Parties as threads of one process, one GPU each: the in-process transport.

``LocalMooseRuntime(..., device_map={identity: device})`` runs every party of an
evaluation as a thread of the calling process, each on its own device and HIP stream,
with the same per-party protocol code as the one-process-per-GPU layout
(:class:`~moose_amd.parallel.spmd.SPMDSession`).  The messages are device-to-device copies
instead of RCCL calls:

* a send copies the payload to the receiver's GPU at once (a peer copy over xGMI, issued
  on the sender's stream) and records an event after it; the receiver's stream waits for
  that event -- no host synchronisation anywhere, so a party's next kernels queue up
  while its messages are in flight, and a receive blocks the receiving thread only until
  the SENDER has issued the copy;
* messages between two parties are FIFO (one queue per ordered pair), which is all the
  per-party protocols need: every party runs the same program in the same order;
* a party that raises marks the hub failed, and every other party blocked on a receive
  raises ``TransportError`` instead of waiting forever.

Reference parity: the reference's ``LocalMooseRuntime`` runs all identities in one
process as async tasks exchanging values through an in-memory networking layer
(``pymoose/src/bindings.rs:137-250``, ``networking/local.rs``); here the identities can
additionally be pinned to different MI355Xs (SURVEY §7.1 "3 parties on 1 or 3 GPUs").
"""
from __future__ import annotations

import functools
import math
import os
import queue
import threading
from typing import Dict
from typing import List
from typing import Optional

import numpy as np
import torch

from moose_amd.ops import ring as R
from moose_amd.parallel.transport import TransportError


def _host(v):
    """A decoded output as something numpy compares (tensors to the host)."""
    return v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else v


def _indexed(d) -> torch.device:
    """``d`` as a torch.device; a bare "cuda" is the current GPU (each party thread sets its
    device, which needs the index)."""
    d = torch.device(d)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


class Hub:
    """The mailboxes of one evaluation's parties (ordered pairs), plus failure state."""

    def __init__(self, devices: List, timeout: Optional[float] = None):
        self.devices = [_indexed(d) for d in devices]
        n = len(self.devices)
        self.boxes = {(s, d): queue.Queue() for s in range(n) for d in range(n) if s != d}
        self.failed: Optional[str] = None
        self.timeout = timeout
        self.lock = threading.Lock()
        self.done = [False] * n  # party i's thread has returned (successfully or not)
        # the baton (BATON): one party thread runs Python at a time and hands over only
        # while it waits for a message -- three threads trading the interpreter lock at
        # every framework call cost each small op several times its own time
        self.baton = threading.Lock() if BATON else None

    def hold(self):
        if self.baton is not None:
            self.baton.acquire()
            self._holder = threading.get_ident()

    def release(self) -> bool:
        """Hand the baton over if this thread holds it; True when it did."""
        if self.baton is None or getattr(self, "_holder", None) != threading.get_ident():
            return False
        self._holder = None
        self.baton.release()
        return True

    def fail(self, why: str):
        with self.lock:
            if self.failed is None:
                self.failed = why

    def finish(self, rank: int):
        self.done[rank] = True


class Mailbox:
    """Messages read where their sender wrote them (the composed one-GPU replay).

    A protocol step that produces a message for another party asks its transport for the
    buffer first (``outbox``; ``SPMDSession.outbox``).  The tapes are captured twice:

    * pass 1 (normal buffers) learns, for every such message, which send it became --
      the k-th tensor from party s to party d is the sender's n-th outbox buffer;
    * pass 2 allocates one persistent buffer per outbox call before capturing again: the
      sender's kernels write the message straight into it, and the receiver -- knowing the
      route -- lands the k-th message in it too.  The message round then needs no copy
      (PartyTapes._compose keeps only a phase boundary).

    Capture is deterministic (same program, same warm-up log), so pass 2 makes the same
    outbox calls and sends in the same order as pass 1."""

    def __init__(self):
        self.pass_ = 1
        self.calls = {}   # (rank, n) -> (shape, dtype) of the n-th outbox request
        self.keep = {}    # pass 1: (rank, n) -> the tensor handed out (kept alive: unique ptr)
        self.by_ptr = {}  # pass 1: data_ptr -> (rank, n)
        self.route = {}   # (src, dst, k) -> n: the k-th message src -> dst is outbox call n
        self.slots = {}   # pass 2: (rank, n) -> persistent buffer

    def prepare(self, device):
        """Pass 2's persistent buffers (before its capture: no allocation inside it)."""
        self.pass_ = 2
        self.keep, self.by_ptr = {}, {}
        routed = {(s, n) for (s, _d, _k), n in self.route.items()}
        for key in sorted(routed):
            shape, dtype = self.calls[key]
            self.slots[key] = torch.empty(shape, dtype=dtype, device=device)
        for key, t in self.slots.items():
            self.by_ptr[t.data_ptr()] = key

    def outbox(self, rank, n, shape, dtype, device):
        shape = tuple(shape)
        if self.pass_ == 1:
            self.calls[(rank, n)] = (shape, dtype)
            t = torch.empty(shape, dtype=dtype, device=device)
            self.keep[(rank, n)] = t
            self.by_ptr[t.data_ptr()] = (rank, n)
            return t
        slot = self.slots.get((rank, n))
        if slot is None or tuple(slot.shape) != shape or slot.dtype != dtype:
            return None  # never sent in pass 1 (or a different request): a normal buffer
        return slot

    def sent(self, rank, dst, k, t):
        """Pass 1: the k-th message rank -> dst was ``t``: an outbox buffer makes a route."""
        key = self.by_ptr.get(t.data_ptr())
        if self.pass_ == 1 and key is not None and key[0] == rank and \
                t.numel() * t.element_size() == self.keep[key].numel() * \
                self.keep[key].element_size():
            self.route[(rank, dst, k)] = key[1]

    def landing(self, src, dst, k, out):
        """Pass 2: the sender's buffer of the k-th message src -> dst (None: a copy)."""
        if self.pass_ != 2:
            return None
        n = self.route.get((src, dst, k))
        slot = self.slots.get((src, n)) if n is not None else None
        if slot is None or slot.numel() != out.numel() or slot.dtype != out.dtype:
            return None
        return slot


class ThreadTransport:
    """Transport API of :class:`~moose_amd.parallel.transport.Transport` (send / recv /
    shift / exchange) between the threads of a :class:`Hub`."""

    plans = False  # no headers: the values themselves travel
    stage = False

    def __init__(self, rank: int, hub: Optional[Hub], device=None, world: Optional[int] = None):
        self.rank, self.hub = rank, hub
        self.world = len(hub.devices) if hub is not None else world
        self.device = hub.devices[rank] if hub is not None else torch.device(device)
        self.bytes_sent = 0
        self.messages = 0
        # what arrived from each peer, in order (kind, shape, dtype, bits): the landing
        # buffers of a taped evaluation are allocated from it (PartyTapes)
        self.log = {}
        # tape mode: every message round goes to this callback as a CommStep
        self.tape = None
        self._cursor = {}
        # per source, the landing buffers of the taped messages allocated OUTSIDE the graph
        # pool (prepare_landing); None: receives land where the protocol allocated them
        self.landing = None
        self._land_cursor = {}
        # messages read where their sender wrote them (Mailbox; composed one-GPU replays)
        self.mailbox = None
        self._outbox_n = 0
        self._send_k, self._recv_k = {}, {}

    def outbox(self, shape, dtype):
        """The buffer of a message this party is about to produce and send (Mailbox), or
        None: the caller allocates it as usual."""
        if self.mailbox is None or self.tape is None:
            return None
        n = self._outbox_n
        self._outbox_n += 1
        return self.mailbox.outbox(self.rank, n, shape, dtype, self.device)

    # -- payload movement --------------------------------------------------------------
    def _ship(self, t: torch.Tensor, dst: int):
        """A private copy of ``t`` on the receiver's device, plus the event it is ready at
        (None on the host)."""
        ddev = self.hub.devices[dst]
        self.bytes_sent += t.numel() * t.element_size()
        self.messages += 1
        if ddev.type != "cuda" and t.device.type != "cuda":
            return t.clone(), None
        # cross-device: a peer copy on this thread's stream of the source device, with
        # PyTorch's two-way barrier against this thread's current stream of ddev, so the
        # event below (on that stream) follows the copy; same device: a clone on our stream
        y = t.to(ddev, copy=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(ddev))
        return y, ev

    def _land(self, y, ev):
        """Make a received copy usable on this thread's stream."""
        if ev is not None:
            s = torch.cuda.current_stream(self.device)
            s.wait_event(ev)
            y.record_stream(s)  # freed only after our stream's use of it
        return y

    def _put(self, dst: int, item):
        if self.hub.failed is not None:
            raise TransportError(f"rank {self.rank}: session failed ({self.hub.failed})")
        self.hub.boxes[(self.rank, dst)].put(item)

    def _get(self, src: int):
        box = self.hub.boxes[(src, self.rank)]
        try:  # already there: no hand-over
            return box.get_nowait()
        except queue.Empty:
            pass
        handed = self.hub.release()  # another party runs while this one waits
        try:
            return self._wait(box, src)
        finally:
            if handed:
                self.hub.hold()

    def _wait(self, box, src: int):
        waited = 0.0
        while True:
            try:
                return box.get(timeout=0.05)
            except queue.Empty:
                waited += 0.05
                if self.hub.failed is not None:
                    raise TransportError(f"rank {self.rank}: no message from rank {src}: "
                                         f"session failed ({self.hub.failed})") from None
                if self.hub.done[src] and box.empty():
                    # the sender returned without sending what this party expects (a
                    # protocol desynchronisation): it never will
                    why = f"rank {src} finished without sending to rank {self.rank}"
                    self.hub.fail(why)
                    raise TransportError(f"rank {self.rank}: {why}") from None
                if self.hub.timeout is not None and waited >= self.hub.timeout:
                    self.hub.fail(f"rank {self.rank} timed out waiting for rank {src}")
                    raise TransportError(f"rank {self.rank}: no message from rank {src} "
                                         f"within {self.hub.timeout} s") from None

    # -- tape mode ------------------------------------------------------------------------
    def prepare_landing(self):
        """Allocate, before a capture, one persistent landing buffer per tensor message of
        the warm-up log.  Needed when a SENDER writes the message into the receiver's memory
        at the sender's own pace (per-party graphs on separate streams / devices): a buffer
        from the receiver's graph pool reuses blocks the receiver's EARLIER segments still
        use (torch reuses pool blocks in the capturing stream's order, which a write from
        another stream does not follow) -- the cause of the composed-as-DAG failures."""
        from moose_amd.ops import native as nat

        self.landing = {}
        for src, items in self.log.items():
            bufs = []
            for kind, shape, dtype, _bits in items:
                if kind in ("rt", "t") and math.prod(shape) > 0:
                    # uncached device memory: the sender's peer writes are what this party's
                    # later kernels read, with no stale line of an earlier replay in its L2
                    bufs.append(nat.uncached_zeros(shape, dtype, self.device)
                                if self.device.type == "cuda" and UNCACHED_LANDING
                                else torch.empty(shape, dtype=dtype, device=self.device))
            self.landing[src] = bufs
        self._land_cursor = {}

    def _take_landing(self, src, out):
        k = self._land_cursor.get(src, 0)
        self._land_cursor[src] = k + 1
        bufs = self.landing.get(src, [])
        if k >= len(bufs) or bufs[k].dtype != out.dtype or bufs[k].numel() != out.numel():
            from moose_amd.runtime.graphs import CaptureError

            raise CaptureError(f"message {k} from rank {src}: no landing buffer of its shape")
        return bufs[k]

    def _taped(self, sends, recvs):
        from moose_amd.parallel.transport import CommStep

        sends = [(t.contiguous(), dst) for t, dst in sends if t.numel()]
        mb = self.mailbox
        for t, dst in sends:
            k = self._send_k.get(dst, 0)
            self._send_k[dst] = k + 1
            if mb is not None:
                mb.sent(self.rank, dst, k, t)
        land, after = [], []
        for out, src in recvs:
            if out.numel() == 0:
                continue
            k = self._recv_k.get(src, 0)
            self._recv_k[src] = k + 1
            slot = mb.landing(src, self.rank, k, out) if mb is not None else None
            if slot is not None:
                if _whole(out) and out.dtype == slot.dtype:
                    out.set_(slot.view(out.shape))  # read where the sender wrote it
                    land.append((slot, src))
                else:  # a view of something larger: copy after the round (own segment)
                    land.append((slot, src))
                    after.append((out, slot))
                continue
            if self.landing is not None:
                buf = self._take_landing(src, out)
                if _whole(out) and tuple(buf.shape) == tuple(out.shape):
                    out.set_(buf)  # the protocol's tensor now IS the persistent buffer
                    land.append((buf, src))
                else:  # a view: land in the persistent buffer, copy after the round
                    land.append((buf, src))
                    after.append((out, buf.view(out.shape) if out.is_contiguous() else buf))
                continue
            if out.is_contiguous():
                land.append((out, src))
            else:
                buf = torch.empty(out.shape, dtype=out.dtype, device=out.device)
                land.append((buf, src))
                after.append((out, buf))
        self.tape(CommStep(sends, land))
        for out, buf in after:  # captured in the segment after the round
            out.copy_(buf.reshape(out.shape))

    def _next_logged(self, src: int):
        k = self._cursor.get(src, 0)
        self._cursor[src] = k + 1
        got = self.log.get(src, [])
        if k >= len(got):
            from moose_amd.runtime.graphs import CaptureError

            raise CaptureError(f"message {k} from rank {src} was not seen in the warm-up")
        return got[k]

    def _logged(self, src: int, item):
        kind, val, _ = item
        if kind == "rt":
            self.log.setdefault(src, []).append(("rt", tuple(val[0].shape), val[0].dtype,
                                                 val[1]))
        elif kind == "t":
            self.log.setdefault(src, []).append(("t", tuple(val.shape), val.dtype, None))
        else:  # a host value (a shape, a scalar): replayed as recorded, like a plan header
            self.log.setdefault(src, []).append(("v", val, None, None))

    # -- typed values ------------------------------------------------------------------
    def send(self, v, dst: int):
        if self.tape is not None:
            if isinstance(v, R.RT):
                v = v.data
            if isinstance(v, torch.Tensor):
                self._taped([(v, dst)], [])
            # a host value (shape, scalar) is not sent: the receiver replays the value it
            # recorded in the warm-up, as Transport replays a message plan's header
            return
        if isinstance(v, R.RT):
            y, ev = self._ship(v.data, dst)
            self._put(dst, ("rt", (y, v.bits), ev))
        elif isinstance(v, torch.Tensor):
            y, ev = self._ship(v, dst)
            self._put(dst, ("t", y, ev))
        else:  # host values (ints, floats, bytes, shapes, None) travel as they are
            self._put(dst, ("v", v, None))

    def recv(self, src: int, device=None):
        if self.tape is not None:
            kind, shape, dtype, bits = self._next_logged(src)
            if kind == "v":
                return shape  # the recorded host value
            buf = torch.empty(shape, dtype=dtype, device=self.device)
            self._taped([], [(buf, src)])
            data = buf if device is None else buf.to(device)
            return R.RT(data, bits) if kind == "rt" else data
        item = self._get(src)
        self._logged(src, item)
        kind, val, ev = item
        if kind == "v":
            return val
        if kind == "rt":
            data, bits = val
            data = self._land(data, ev)
            return R.RT(data if device is None else data.to(device), bits)
        data = self._land(val, ev)
        return data if device is None else data.to(device)

    # -- structured exchanges ------------------------------------------------------------
    def shift(self, t: torch.Tensor, to_rank: int, from_rank: int) -> torch.Tensor:
        if t.numel() == 0:
            return torch.empty_like(t)
        if self.tape is not None:
            t = t.contiguous()
            out = torch.empty_like(t)
            self._next_logged(from_rank)
            self._taped([(t, to_rank)], [(out, from_rank)])
            return out
        self.send(t, to_rank)
        return self.recv(from_rank)

    def exchange(self, sends, recvs):
        """Sends first (they never block), then each receive lands in its buffer."""
        if self.tape is not None:
            for out, src in recvs:
                if out.numel():
                    self._next_logged(src)
            self._taped(sends, recvs)
            return
        for t, dst in sends:
            if t.numel():
                self.send(t, dst)
        for out, src in recvs:
            if out.numel():
                y = self.recv(src)
                if isinstance(y, R.RT):
                    y = y.data
                if (_whole(out) and y.device == out.device and y.dtype == out.dtype
                        and y.numel() == out.numel() and y.is_contiguous()):
                    # the received tensor is a private copy already: adopt its storage
                    # instead of copying it once more
                    out.set_(y.view(out.shape))
                else:
                    out.copy_(y.reshape(out.shape))

    def end_evaluation(self):
        pass

    def broadcast_from(self, v, src: int, dsts: List[int], me: int):
        if me == src:
            for d in dsts:
                if d != src:
                    self.send(v, d)
            return v
        if me in dsts:
            return self.recv(src)
        return None


# a party that waits this long for a message ends the evaluation (device_map runtimes
# without an explicit timeout); a desynchronised peer that returned is detected at once
DEFAULT_TIMEOUT_S = float(os.environ.get("MOOSEX_PARTY_TIMEOUT", "300"))
# segments per composed executable (0: the whole tape is ONE executable; > 0: a larger tape
# is replayed as several, back to back).  Round 5 chunked at 200 against a crash that was
# the flattening of captured copy nodes, not the graph's size
# (profiles/r6_graph_flatten_segfault.md): a 100-iteration LogReg tape is one 28,512-node
# executable
CHUNK_SEGMENTS = int(os.environ.get("MOOSEX_PARTY_GRAPH_CHUNK", "0"))
# per-party stream graphs: message flags and landing buffers in uncached device memory
# (MOOSEX_PARTY_UNCACHED=0: PyTorch's allocator, coarse-grained -- probes only)
UNCACHED_LANDING = os.environ.get("MOOSEX_PARTY_UNCACHED", "1") != "0"
# per-party stream graphs are checked once at capture against the per-action replay of the
# same tapes from the same key state (bitwise); a mismatch keeps the per-action replay
VALIDATE_STREAMS = os.environ.get("MOOSEX_PARTY_STREAMS_VALIDATE", "1") != "0"
# the composed one-GPU graph as a DAG (each party's nodes in program order, a message copy
# after its sender's segment and before its receiver's next one, and the sender's next
# segment after the copy has read its buffer) instead of one total order: the parties'
# branches may run concurrently inside the one launch.  Needs persistent landing buffers
# (ThreadTransport.prepare_landing; profiles/r5_party_dag_hazard.md)
DAG_COMPOSE = os.environ.get("MOOSEX_PARTY_GRAPH_DAG", "0") == "1"
# composed one-GPU replays: messages read where their senders wrote them (Mailbox)
INPLACE = os.environ.get("MOOSEX_PARTY_INPLACE", "1") != "0"
# in-process parties run their Python one at a time, handing over while they wait for a
# message (Hub.baton; MOOSEX_PARTY_BATON=0: free-running threads)
BATON = os.environ.get("MOOSEX_PARTY_BATON", "1") != "0"
# the composed chain batches the same launch of several parties into one node
# (csrc/party_batch.h; MOOSEX_PARTY_MERGE=0: one node per launch)
MERGE_PARTIES = os.environ.get("MOOSEX_PARTY_MERGE", "1") != "0"


def _whole(t: torch.Tensor) -> bool:
    """``t`` is its storage's only view (not a slice or view of a larger tensor)."""
    return (t._base is None and t.storage_offset() == 0 and t.is_contiguous()
            and t.untyped_storage().nbytes() == t.numel() * t.element_size())


def _touch(dst: int, src: int) -> int:
    """The parties a message copy writes to and reads from, as a bitmask (every party when
    one is beyond the third): the composed graph's merging keeps each party's launches
    on their side of every copy that touches the party (csrc/graph_compose.hip)."""
    return 7 if dst > 2 or src > 2 else (1 << dst) | (1 << src)


def chunk_bounds(kinds, per: int):
    """[(start, end)) node ranges of a composed schedule, each holding at most ``per``
    segment nodes (kind 0); a chunk starts at a segment, so the copies after a chunk's last
    segment stay in that chunk."""
    bounds, start, nseg = [], 0, 0
    for i, k in enumerate(kinds):
        if k == 0:
            if nseg == per:
                bounds.append((start, i))
                start, nseg = i, 0
            nseg += 1
    bounds.append((start, len(kinds)))
    return bounds


class _Workers:
    """Party threads kept between evaluations: starting three threads per evaluation cost
    ~0.8 ms of an eager one (the interpreter bootstraps each while the parties run).  A
    worker runs one party at a time under that party's thread name; a worker still busy
    (a party that never returned) is simply not reused -- a new one starts."""

    def __init__(self):
        self._idle = queue.SimpleQueue()

    def run(self, fn, name: str) -> threading.Event:
        done = threading.Event()
        try:
            inbox = self._idle.get_nowait()
        except queue.Empty:
            inbox = queue.SimpleQueue()
            threading.Thread(target=self._loop, args=(inbox,), name=name, daemon=True).start()
        inbox.put((fn, name, done))
        return done

    def _loop(self, inbox):
        while True:
            fn, name, done = inbox.get()
            threading.current_thread().name = name
            try:
                fn()
            finally:
                done.set()
                self._idle.put(inbox)


_WORKERS = _Workers()


def run_parties(comp, arguments: dict, identities: List[str], devices: List, storage: dict,
                fixedpoint_ring: int = 128, seed: Optional[int] = None,
                timeout: Optional[float] = None, record: bool = False):
    """Evaluate ``comp`` with party ``identities[i]`` as a thread on ``devices[i]``.
    Returns ``(outputs, stats_by_identity, elapsed_us_by_identity, warm)``: the outputs of
    every party merged (each output tag is materialised by the party that owns it);
    ``warm`` (with ``record``) holds per party what a :class:`PartyTapes` capture needs
    -- the uploads, the first outputs, the stats, the key slots used and the message log."""
    import time

    from moose_amd.compiler.passes import is_lowered
    from moose_amd.parallel.spmd import SPMDSession
    from moose_amd.runtime import graphs as G
    from moose_amd.runtime.interpreter import Interpreter

    hub = Hub(devices, timeout=DEFAULT_TIMEOUT_S if timeout is None else timeout)
    role_ranks = {r: i for i, r in enumerate(identities)}
    results, stats, elapsed, errors, warm = {}, {}, {}, {}, {}
    lowered = is_lowered(comp)

    def party(i):
        ident, dev = identities[i], hub.devices[i]
        tr = ThreadTransport(i, hub)
        rec = None
        hub.hold()
        try:
            if record:  # this thread's host->device copies go to its recorder
                rec = G._Recorder()
                R.set_upload_hook(rec)
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
                stream = torch.cuda.Stream(dev)
                ctx = torch.cuda.stream(stream)
            else:
                import contextlib

                ctx = contextlib.nullcontext()
            t0 = time.perf_counter()
            with ctx:
                if lowered:
                    from moose_amd.runtime.distributed import _host_numpy
                    from moose_amd.runtime.graph_executor import GraphExecutor

                    ex = GraphExecutor(dev, storage, identity=ident, transport=tr,
                                       role_ranks=role_ranks)
                    raw = ex.run(comp, arguments)
                    out = {k: _host_numpy(v) for k, v in raw.items()}
                    st = None
                else:
                    sess = SPMDSession(ident, role_ranks, tr, device=dev, seed=seed)
                    interp = Interpreter(sess, storage, fixedpoint_ring)
                    outs = interp.run(comp, arguments)
                    out = {tag: interp.to_numpy(lv) for tag, lv in outs.items()
                           if lv.kind != "unit" and sess.materialized(lv.v)}
                    st = sess.stats
                    if rec is not None:
                        warm[ident] = {"uploads": rec.items, "first": out, "stats": st,
                                       "keys_n": sess.keytable.n, "log": tr.log}
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            elapsed[ident] = int((time.perf_counter() - t0) * 1e6)
            results[ident], stats[ident] = out, st
        except BaseException as e:  # noqa: BLE001 - reported after every party stopped
            errors[ident] = e
            hub.fail(f"{ident}: {type(e).__name__}: {e}")
        finally:
            if rec is not None:
                R.set_upload_hook(None)
            hub.finish(i)
            hub.release()

    R.shared_streams(+1)  # shared device constants: their producer drains first
    try:
        names = [f"moose-party-{identities[i]}" for i in range(len(identities))]
        done = [_WORKERS.run(functools.partial(party, i), names[i])
                for i in range(len(identities))]
        for name, ev in zip(names, done):
            # every blocked receive gives up within the hub's timeout (or at once when its
            # sender has returned), so the waits end; the bound is a last resort
            if not ev.wait(hub.timeout + 60.0):
                hub.fail(f"{name} did not finish")
                raise TransportError(f"{name} did not finish within {hub.timeout + 60.0} s")
    finally:
        R.shared_streams(-1)
    if errors:
        # the first party to fail is the cause; the others saw TransportError because of it
        first = next((e for e in errors.values() if not isinstance(e, TransportError)),
                     next(iter(errors.values())))
        raise first
    merged = {}
    for ident in identities:
        merged.update(results[ident])
    return merged, stats, elapsed, (warm if record and not lowered else None)


class PartyTapes:
    """Replayed evaluations of the in-process parties: one recorded tape per party
    (parallel/spmd_graphs.SPMDTape: hipGraph segments between message rounds, captured on
    the party's own device), replayed by ONE host thread that interleaves the parties.

    At capture the rounds of all tapes are matched (the k-th message from party a to b is
    the k-th receive at b from a) and turned into a fixed issue order: a party's segments
    run until a round that receives something whose sender has not been issued yet, then
    another party goes on.  A send records an event on the sender's stream; the receiver's
    stream waits for it and copies into its landing buffer (a peer copy over xGMI from a
    copy stream of the source GPU when the parties are on different devices), so every
    dependency is a stream/event edge and the host never waits inside a replay."""

    def __init__(self, comp, arguments: dict, identities: List[str], devices: List,
                 storage: dict, ring: int, seed: Optional[int], warm: dict):
        from moose_amd.parallel.spmd_graphs import SPMDTape

        self.identities = list(identities)
        self.devices = [_indexed(d) for d in devices]
        n = len(identities)
        role_ranks = {r: i for i, r in enumerate(identities)}
        # every party on one device: the tapes are composed into ONE graph (below)
        # per-party graphs on their own streams / devices with device-side message flags
        # (_build_streams): the default when the parties are on several devices (one GPU:
        # the composed graph, unless MOOSEX_PARTY_STREAMS=1; =0 disables it everywhere)
        env = os.environ.get("MOOSEX_PARTY_STREAMS")
        self.streams_mode = env == "1" or (env is None and len(set(self.devices)) > 1)
        single = (len(set(self.devices)) == 1 and not self.streams_mode
                  and os.environ.get("MOOSEX_PARTY_GRAPH", "1") != "0")
        # the composed graph runs every party on one stream: the tapes share their argument
        # buffers, uploaded once per replay
        self.shared_static = single and not DAG_COMPOSE
        # ... and read their messages where the senders wrote them (Mailbox: two capture
        # passes; MOOSEX_PARTY_INPLACE=0: every message copied)
        mailbox = Mailbox() if (self.shared_static and INPLACE and MERGE_PARTIES
                                and CHUNK_SEGMENTS <= 0) else None

        def capture():
            tapes, shared = [], {}
            for i, ident in enumerate(identities):
                tr = ThreadTransport(i, None, device=self.devices[i], world=n)
                tr.log = warm[ident]["log"]
                tr.mailbox = mailbox
                if self.streams_mode or (DAG_COMPOSE and len(set(self.devices)) == 1):
                    # senders write landing buffers at their own pace (streams), or a copy
                    # runs when its sender's branch reaches it (DAG): persistent buffers
                    with torch.cuda.device(self.devices[i]):
                        tr.prepare_landing()
                with torch.cuda.device(self.devices[i]):
                    tapes.append(SPMDTape(comp, arguments, ident, role_ranks, tr,
                                          self.devices[i], storage, ring, seed,
                                          warm=warm[ident],
                                          keep_graph=single or self.streams_mode,
                                          shared_static=shared.setdefault(
                                              self.devices[i], {})
                                          if self.shared_static else None))
            return tapes

        self.tapes = capture()
        self.inplace_messages = 0
        if mailbox is not None and mailbox.route:
            # pass 2: the routed outbox buffers exist before the capture, senders write
            # their messages into them and receivers read them there
            self.tapes = None
            torch.cuda.synchronize(self.devices[0])
            mailbox.prepare(self.devices[0])
            self.tapes = capture()
            self.inplace_messages = len(mailbox.route)
        self._mailbox = mailbox  # the persistent message buffers live with the graphs
        self.streams = [t.stream for t in self.tapes]
        self._copy_streams = {}
        self.actions = self._schedule()
        self.rounds = max(t.rounds for t in self.tapes)
        self.segments = sum(t.segments for t in self.tapes)
        self._ends = None
        self.issue_s = []
        self.issue_parts = []
        self._composed = self._compose() if single else None
        self._party_graphs = None
        self._launchers = None  # host threads issuing the per-party graph launches
        # how replays run, and whether the per-party graphs were checked at capture
        self.validated = None
        self.fallback = None
        if self.streams_mode:
            try:
                self._party_graphs = self._build_streams()
            except Exception as e:  # noqa: BLE001 - e.g. no peer access between the GPUs
                import warnings

                self.fallback = f"per-party stream graphs unavailable: {e}"
                warnings.warn(f"{self.fallback}; per-action replay", RuntimeWarning,
                              stacklevel=2)
            if self._party_graphs is not None and VALIDATE_STREAMS:
                self._validate_streams(arguments)

    @property
    def replay_form(self) -> str:
        if self._party_graphs is not None:
            return "party_graphs"
        return "composed" if self._composed is not None else "per_action"

    def _key_state(self):
        """Each tape's device key-refresh counter (unseeded tapes draw replay e's keys from
        ChaCha12(master, e)): saved and restored around a validation replay so the
        per-action replay runs from the same keys."""
        return [t.keys._epoch.clone() if getattr(t.keys, "_epoch", None) is not None else None
                for t in self.tapes]

    def _set_key_state(self, state):
        for t, e in zip(self.tapes, state):
            if e is not None:
                t.keys._epoch.copy_(e)

    def _validate_streams(self, arguments: dict):
        """Run the per-party graphs once and the per-action replay of the same tapes once,
        from the same key state and arguments, and compare every party's outputs bitwise.
        The per-action replay orders every message with stream events (no flags, no peer
        writes of our own): if the graphs' device-side messaging misbehaves on this machine
        (a lost or stale push, a flag seen before its payload), the outputs differ and the
        runtime keeps the per-action replay -- recorded in ``fallback`` / ``validated`` --
        instead of returning wrong values later."""
        import warnings

        from moose_amd.parallel.transport import TransportError

        for d in set(self.devices):
            torch.cuda.synchronize(d)
        state = self._key_state()
        why = None
        try:
            got = self._replay_streams(arguments)
        except TransportError as e:
            got, why = None, f"a message never arrived ({e})"
        for d in set(self.devices):
            torch.cuda.synchronize(d)
        for err in self._errs:
            err.zero_()
        self._set_key_state(state)
        want = self._replay_actions(arguments)
        for d in set(self.devices):
            torch.cuda.synchronize(d)
        for t in self.tapes:
            t.replays -= 2  # the two validation replays are not evaluations
        if got is not None:
            for ident in self.identities:
                a, b = got.get(ident, {}), want.get(ident, {})
                if set(a) != set(b) or any(
                        not np.array_equal(np.asarray(_host(a[k])), np.asarray(_host(b[k])))
                        for k in a):
                    why = f"outputs of {ident} differ from the per-action replay"
                    break
        if why is None:
            self.validated = True
            return
        self.validated = False
        self.fallback = f"per-party stream graphs failed validation: {why}"
        warnings.warn(f"{self.fallback}; per-action replay", RuntimeWarning, stacklevel=3)
        self._free_party_graphs()

    def _compose(self):
        """The schedule as ONE hipGraph (csrc/graph_compose.hip) in a total order: each
        segment a child graph; the messages of one round of all parties ONE batched copy
        kernel (csrc/party_graph.hip k_copy_many; ``MOOSEX_PARTY_COPY_BATCH=0``: a copy node
        per message).  None when the runtime declines (the per-action replay is used)."""
        import ctypes

        from moose_amd.ops import native as nat

        if DAG_COMPOSE:
            return self._compose_dag()
        batched = os.environ.get("MOOSEX_PARTY_COPY_BATCH", "1") != "0"
        acts = self._schedule_rounds() if batched else [
            a if a[0] != "cp" else ("cpb", [(a[1], a[2], a[3], a[4])])
            for a in self.actions if a[0] != "rec"]
        # the device key refresh of unseeded tapes as the head of the graph (one captured
        # launch per party, batched into one node) instead of a host launch per replay
        keyg = {p: g for p, g in ((p, self._key_graph(t)) for p, t in enumerate(self.tapes))
                if g is not None} if batched and MERGE_PARTIES else {}
        acts = [("g", p, g) for p, g in keyg.items()] + acts
        # the argument uploads (pinned staging -> static buffer) as the graph's first
        # nodes: a replay only stages the new values on the host
        ups = [(t, pin) for tape in self.tapes for t, pin in tape.uploads()] \
            if batched and MERGE_PARTIES and CHUNK_SEGMENTS <= 0 else []
        kinds, child, dst, src, nbytes, party = [], [], [], [], [], []
        for t, pin in ups:
            kinds.append(3)
            child.append(0)
            dst.append(t.data_ptr())
            src.append(pin.data_ptr())
            nbytes.append(t.numel() * t.element_size())
            party.append(7)
        descs = []
        for a in acts:
            if a[0] == "g":
                kinds.append(0)
                party.append(a[1])
                child.append(a[2].raw_cuda_graph())
                dst.append(0)
                src.append(0)
                nbytes.append(0)
                continue
            mask = 0
            for _p, _s, _t, _b in a[1]:
                mask |= _touch(_p, _s)
            # a message read where its sender wrote it (Mailbox) needs no copy; a round of
            # only such messages is a phase boundary (kind 4, no node)
            msgs = [m for m in a[1] if m[2].data_ptr() != m[3].data_ptr()]
            if not msgs:
                kinds.append(4)
                party.append(mask)
                child.append(0)
                dst.append(0)
                src.append(0)
                nbytes.append(0)
                continue
            if len(msgs) == 1 or not batched:
                for _p, _s, t, buf in msgs:
                    kinds.append(1)
                    party.append(_touch(_p, _s))
                    child.append(0)
                    dst.append(buf.data_ptr())
                    src.append(t.data_ptr())
                    nbytes.append(t.numel() * t.element_size())
                continue
            descs.append([(t.data_ptr(), buf.data_ptr(), t.numel() * t.element_size())
                          for _p, _s, t, buf in msgs])
            kinds.append(2)
            party.append(mask)
            child.append(len(msgs))
            dst.append(len(descs) - 1)  # the table's address is filled in below
            src.append(0)
            nbytes.append(max(b for _, _, b in descs[-1]))
        if descs:
            flat = [v for d in descs for e in d for v in e]
            table = torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in flat],
                                 dtype=torch.int64, device=self.devices[0])
            self._copy_table = table  # alive as long as the graph
            offs, at = [], 0
            for d in descs:
                offs.append(table.data_ptr() + 8 * 3 * at)
                at += len(d)
            dst = [offs[d] if k == 2 else d for k, d in zip(kinds, dst)]
        arr = lambda ty, xs: (ty * max(1, len(xs)))(*xs)  # noqa: E731
        if batched and CHUNK_SEGMENTS <= 0 and MERGE_PARTIES:
            # one chain in which the same launch of 2-3 parties between two rounds is ONE
            # party-batched node (csrc/party_batch.h)
            g, ex = ctypes.c_void_p(), ctypes.c_void_p()
            st = (ctypes.c_int64 * 4)()
            rc = nat.lib().mx_graph_compose_merged(
                len(kinds), arr(ctypes.c_int, kinds), arr(ctypes.c_void_p, child),
                arr(ctypes.c_void_p, dst), arr(ctypes.c_void_p, src),
                arr(ctypes.c_int64, nbytes), arr(ctypes.c_int, party), st, ctypes.byref(g),
                ctypes.byref(ex))
            if rc == 0:
                self._uploads_in_graph = bool(ups)
                self._keys_in_graph = set(keyg)
                self._key_graphs = keyg  # alive as long as the composed graph
                self._graph_handles = [(g, ex)]
                self.graph_nodes = {"segments": kinds.count(0), "copy_nodes": kinds.count(1),
                                    "copy_batches": kinds.count(2), "executables": 1,
                                    "inplace_rounds": kinds.count(4),
                                    "inplace_messages": self.inplace_messages,
                                    "nodes": st[0], "merged_away": st[1],
                                    "party_batched": st[2], "phases": st[3]}
                return [ex]
        if keyg or ups:  # not composed with the merged chain: the host does these
            kinds, child, dst, src, nbytes, party = (
                xs[len(ups) + len(keyg):] for xs in (kinds, child, dst, src, nbytes, party))
        keep = [i for i, k in enumerate(kinds) if k != 4]  # a plain chain needs no boundary
        kinds, child, dst, src, nbytes, party = (
            [xs[i] for i in keep] for xs in (kinds, child, dst, src, nbytes, party))
        # the total order as one executable, or in chunks of at most CHUNK_SEGMENTS
        # segments launched back to back on one stream
        bounds = (chunk_bounds(kinds, CHUNK_SEGMENTS) if CHUNK_SEGMENTS > 0
                  else [(0, len(kinds))])
        handles = []
        for a, b in bounds:
            m = b - a
            off = [0] + [max(0, i) for i in range(m)]  # node i > 0 waits for node i - 1
            flat_deps = list(range(m - 1))
            g, ex = ctypes.c_void_p(), ctypes.c_void_p()
            rc = nat.lib().mx_graph_compose(
                m, arr(ctypes.c_int, kinds[a:b]), arr(ctypes.c_void_p, child[a:b]),
                arr(ctypes.c_void_p, dst[a:b]), arr(ctypes.c_void_p, src[a:b]),
                arr(ctypes.c_int64, nbytes[a:b]), arr(ctypes.c_int, off),
                arr(ctypes.c_int, flat_deps), ctypes.byref(g), ctypes.byref(ex))
            if rc != 0:
                for gh, eh in handles:
                    nat.lib().mx_graph_free(gh, eh)
                return None
            handles.append((g, ex))
        self._graph_handles = handles
        self.graph_nodes = {"segments": kinds.count(0), "copy_nodes": kinds.count(1),
                            "copy_batches": kinds.count(2), "executables": len(handles)}
        return [ex for _, ex in handles]

    def _key_graph(self, tape):
        """The unseeded tape's device key refresh (runtime/keys.py refresh_device: the
        replay counter lives in device memory, so a captured launch draws fresh keys at
        every replay) captured on the tape's stream; None for seeded tapes."""
        keys = tape.keys
        if tape.seed is not None or getattr(keys, "_master", None) is None:
            return None
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.device(tape.device), torch.cuda.stream(tape.stream):
            g.capture_begin(capture_error_mode="thread_local")
            try:
                keys.refresh_device(keys.n)
            finally:
                g.capture_end()
        return g

    def _compose_dag(self):
        """The per-action schedule as ONE graph with only the protocol's edges
        (MOOSEX_PARTY_GRAPH_DAG=1): a party's segments and receive copies in its program
        order, a copy after the sender's segment that produced the message, and the sender's
        next segment after every copy that read its buffer (write-after-read).  Returns
        [exec] or None when the runtime declines."""
        import ctypes

        from moose_amd.ops import native as nat

        n = len(self.tapes)
        kinds, child, dst, src, nbytes, deps = [], [], [], [], [], []
        last = [None] * n
        sent_at = {}
        reading = [[] for _ in range(n)]
        for a in self.actions:
            p = a[1]
            if a[0] == "g":
                kinds.append(0)
                child.append(a[2].raw_cuda_graph())
                dst.append(0)
                src.append(0)
                nbytes.append(0)
                deps.append(sorted(set(([last[p]] if last[p] is not None else []) +
                                       reading[p])))
                reading[p] = []
                last[p] = len(kinds) - 1
            elif a[0] == "rec":
                sent_at[id(a[2])] = (last[p], p)
            else:
                _, p, _s, t, buf, ev = a
                at, sender = sent_at.get(id(ev), (None, None))
                kinds.append(1)
                child.append(0)
                dst.append(buf.data_ptr())
                src.append(t.data_ptr())
                nbytes.append(t.numel() * t.element_size())
                deps.append(sorted(set(x for x in (last[p], at) if x is not None)))
                last[p] = len(kinds) - 1
                if sender is not None and sender != p:
                    reading[sender].append(last[p])
        off, flat = [0], []
        for d in deps:
            flat += d
            off.append(len(flat))
        arr = lambda ty, xs: (ty * max(1, len(xs)))(*xs)  # noqa: E731
        g, ex = ctypes.c_void_p(), ctypes.c_void_p()
        rc = nat.lib().mx_graph_compose(
            len(kinds), arr(ctypes.c_int, kinds), arr(ctypes.c_void_p, child),
            arr(ctypes.c_void_p, dst), arr(ctypes.c_void_p, src), arr(ctypes.c_int64, nbytes),
            arr(ctypes.c_int, off), arr(ctypes.c_int, flat), ctypes.byref(g), ctypes.byref(ex))
        if rc != 0:
            return None
        self._graph_handles = [(g, ex)]
        self.graph_nodes = {"segments": kinds.count(0), "copy_nodes": kinds.count(1),
                            "copy_batches": 0, "executables": 1, "dag": True}
        return [ex]

    def _build_streams(self):
        """Every party's replay as ONE graph on its own stream (its own GPU when the parties
        are on several): its segments in program order and, at each message round, a PUSH
        node -- the round's payloads copied into the receivers' landing buffers (peer writes
        over xGMI across GPUs), then each message's flag raised to the replay number -- and a
        WAIT node for the flags of the round's receives (csrc/party_graph.hip).  The graphs
        depend on each other only through the flags in device memory, so they are launched
        independently (no host issue per message, no launch order) and run concurrently.
        Returns the per-party (graph, exec) handles, or None when the runtime declines."""
        import ctypes

        from moose_amd.ops import native as nat
        from moose_amd.parallel.transport import CommStep

        n = len(self.tapes)
        # the k-th message from party a to party b is the k-th receive at b from a
        land, flag_of, nflags = {}, {}, [0] * n
        for q, tape in enumerate(self.tapes):
            cnt = {}
            for st in tape.steps:
                if isinstance(st, CommStep):
                    for buf, src in st.recvs:
                        k = cnt.get(src, 0)
                        cnt[src] = k + 1
                        land[(src, q, k)] = buf
                        flag_of[(src, q, k)] = nflags[q]
                        nflags[q] += 1
        for p in range(n):
            for q in range(n):
                if p != q and self.devices[p] != self.devices[q]:
                    nat.check(nat.lib().mx_enable_peer(self.devices[p].index,
                                                       self.devices[q].index), "peer access")
        # the flags a peer raises while this party polls: uncached device memory (coherent
        # without kernel boundaries; csrc/party_graph.hip mx_alloc_uncached)
        self._flags = [nat.uncached_zeros((max(1, nflags[q]),), torch.int32, self.devices[q])
                       if UNCACHED_LANDING else
                       torch.zeros(max(1, nflags[q]), dtype=torch.int32, device=self.devices[q])
                       for q in range(n)]
        self._epochs = [torch.zeros(1, dtype=torch.int64, device=d) for d in self.devices]
        self._errs = [torch.zeros(1, dtype=torch.int32, device=d) for d in self.devices]
        self._tables = []
        # MOOSEX_PARTY_STREAMS_SHADOW=1 (probes): copies of the landing buffers after waits
        shadow = os.environ.get("MOOSEX_PARTY_STREAMS_SHADOW") == "1"
        self._shadows = []
        self._dummy = torch.zeros(64, dtype=torch.int32, device=self.devices[0])
        # test-only fault injection (MOOSEX_FAULT=party_landing): the first push writes a
        # scratch buffer instead of its receiver's landing buffer -- the receiver reads a
        # stale message, which the capture-time validation must catch
        fault = os.environ.get("MOOSEX_FAULT") == "party_landing"
        handles = []
        for p, tape in enumerate(self.tapes):
            dev = self.devices[p]
            kinds, child, p0, p1, p2, i0, i64 = [], [], [], [], [], [], []

            def node(kind, ch=0, a=0, b=0, c=0, cnt=0, big=0):
                kinds.append(kind)
                child.append(ch)
                p0.append(a)
                p1.append(b)
                p2.append(c)
                i0.append(cnt)
                i64.append(big)

            epoch = self._epochs[p].data_ptr()
            node(5, a=epoch)
            sent = {}
            fbase = 0
            for st in tape.steps:
                if not isinstance(st, CommStep):
                    node(0, ch=st.raw_cuda_graph())
                    continue
                if st.sends:
                    rows = []
                    pieces = torch.zeros(len(st.sends), dtype=torch.int32, device=dev)
                    for j, (t, dst) in enumerate(st.sends):
                        k = sent.get(dst, 0)
                        sent[dst] = k + 1
                        buf = land[(p, dst, k)]
                        if t.numel() != buf.numel() or t.dtype != buf.dtype:
                            from moose_amd.runtime.graphs import CaptureError

                            raise CaptureError(f"message {k} from party {p} to {dst}: sizes "
                                               "differ")
                        flag = self._flags[dst].data_ptr() + 4 * flag_of[(p, dst, k)]
                        if fault:
                            fault = False
                            buf = torch.empty_like(buf)
                            self._tables.append(buf)
                        rows.append((t.data_ptr(), buf.data_ptr(),
                                     t.numel() * t.element_size(), flag,
                                     pieces.data_ptr() + 4 * j))
                    flat = [x - (1 << 64) if x >= (1 << 63) else x for r in rows for x in r]
                    table = torch.tensor(flat, dtype=torch.int64, device=dev)
                    self._tables += [table, pieces]
                    node(6, a=table.data_ptr(), b=epoch, cnt=len(rows),
                         big=max(r[2] for r in rows))
                if st.recvs:
                    node(7, a=self._flags[p].data_ptr() + 4 * fbase, b=epoch,
                         c=self._errs[p].data_ptr(), cnt=len(st.recvs))
                    fbase += len(st.recvs)
                    if shadow:  # debugging: each landing buffer as seen right after the wait
                        rows = []
                        for buf, _src in st.recvs:
                            sh = torch.empty_like(buf)
                            self._shadows.append((buf, sh))
                            rows.append((buf.data_ptr(), sh.data_ptr(),
                                         buf.numel() * buf.element_size(),
                                         self._dummy.data_ptr(), self._dummy.data_ptr() + 4))
                        flat = [x - (1 << 64) if x >= (1 << 63) else x for r in rows for x in r]
                        table = torch.tensor(flat, dtype=torch.int64, device=dev)
                        self._tables.append(table)
                        node(6, a=table.data_ptr(), b=epoch, cnt=len(rows),
                             big=max(r[2] for r in rows))
            m = len(kinds)
            arr = lambda ty, xs: (ty * max(1, len(xs)))(*xs)  # noqa: E731
            g, ex = ctypes.c_void_p(), ctypes.c_void_p()
            with torch.cuda.device(dev):
                rc = nat.lib().mx_graph_build_chain(
                    m, arr(ctypes.c_int, kinds), arr(ctypes.c_void_p, child),
                    arr(ctypes.c_void_p, p0), arr(ctypes.c_void_p, p1), arr(ctypes.c_void_p, p2),
                    arr(ctypes.c_int, i0), arr(ctypes.c_int64, i64), ctypes.byref(g),
                    ctypes.byref(ex))
            if rc != 0:
                for gh, eh in handles:
                    nat.lib().mx_graph_free(gh, eh)
                import warnings

                warnings.warn(f"per-party graph of party {p} not built (mx_graph_build_chain "
                              f"{rc}); per-action replay", RuntimeWarning, stacklevel=2)
                return None
            handles.append((g, ex))
        self.graph_nodes = {"per_party_nodes": [len(t.steps) for t in self.tapes]}
        return handles

    def _replay_streams(self, arguments: dict) -> Dict[str, dict]:
        """One graph launch per party on its own stream, after its arguments and keys."""
        import time

        from moose_amd.ops import native as nat

        def launch(p):
            tape, s = self.tapes[p], self.streams[p]
            with torch.cuda.device(self.devices[p]), torch.cuda.stream(s):
                tape.copy_arguments(arguments)
                tape._fill_keys()
                nat.check(nat.lib().mx_graph_launch(self._party_graphs[p][1], s.cuda_stream),
                          "party graph launch")

        t0 = time.perf_counter()
        if self._launchers is None and os.environ.get("MOOSEX_PARTY_LAUNCH_THREADS",
                                                      "1") != "0":
            from concurrent.futures import ThreadPoolExecutor

            self._launchers = ThreadPoolExecutor(len(self.tapes) - 1,
                                                 thread_name_prefix="moose-party-launch")
        if self._launchers is not None:
            # hipGraphLaunch enqueues every node from the host: the parties' launches go out
            # concurrently, so a party's graph does not wait behind another's enqueue (its
            # first receive would otherwise stall until then)
            futs = [self._launchers.submit(launch, p) for p in range(1, len(self.tapes))]
            launch(0)
            for f in futs:
                f.result()
        else:
            for p in range(len(self.tapes)):
                launch(p)
        self.issue_s.append(time.perf_counter() - t0)
        out = {}
        for p, tape in enumerate(self.tapes):
            with torch.cuda.device(self.devices[p]), torch.cuda.stream(self.streams[p]):
                out[self.identities[p]] = tape._decode(tape.interp, tape.sess, tape.outs)
                tape.replays += 1
        for p in range(len(self.tapes)):
            self.streams[p].synchronize()
        errs = [int(e.item()) for e in self._errs]
        if any(errs):
            from moose_amd.parallel.transport import TransportError

            raise TransportError(f"party graphs: a message never arrived (flags {errs}); the "
                                 "replay is void")
        return out

    def _schedule_rounds(self):
        """The tapes as a round-synchronous total order: every party runs its segments up to
        its next round, then the messages of all parties whose round can complete (every
        sender has reached it) are copied together -- one batch per round instead of one
        copy per message (the composed one-GPU replay).  Returns ("g", party, graph) and
        ("cpb", [(receiver, sender, payload, landing buffer)]) actions."""
        from moose_amd.parallel.transport import CommStep
        from moose_amd.runtime.graphs import CaptureError

        n = len(self.tapes)
        steps = [t.steps for t in self.tapes]
        ptr, sent_done = [0] * n, [False] * n
        sent, recvd, pending = {}, {}, {}
        acts = []
        while any(ptr[p] < len(steps[p]) for p in range(n)):
            progress = False
            for p in range(n):  # every party up to its next round; its sends go out
                while ptr[p] < len(steps[p]) and not isinstance(steps[p][ptr[p]], CommStep):
                    acts.append(("g", p, steps[p][ptr[p]]))
                    ptr[p] += 1
                    progress = True
                if ptr[p] < len(steps[p]) and not sent_done[p]:
                    for t, dst in steps[p][ptr[p]].sends:
                        k = sent.get((p, dst), 0)
                        sent[(p, dst)] = k + 1
                        pending[(p, dst, k)] = t
                    sent_done[p] = True
                    progress = True
            batch = []
            for p in range(n):  # every round whose messages have all been sent completes
                if ptr[p] >= len(steps[p]) or not sent_done[p]:
                    continue
                s = steps[p][ptr[p]]
                need = {}
                for _, src in s.recvs:
                    need[src] = need.get(src, 0) + 1
                if any(sent.get((src, p), 0) < recvd.get((src, p), 0) + c
                       for src, c in need.items()):
                    continue
                for buf, src in s.recvs:
                    k = recvd.get((src, p), 0)
                    recvd[(src, p)] = k + 1
                    t = pending.pop((src, p, k))
                    if t.numel() != buf.numel() or t.dtype != buf.dtype:
                        raise CaptureError(f"message {k} from party {src} to {p}: "
                                           f"{tuple(t.shape)} {t.dtype} sent, "
                                           f"{tuple(buf.shape)} {buf.dtype} expected")
                    batch.append((p, src, t.reshape(buf.shape), buf))
                ptr[p] += 1
                sent_done[p] = False
                progress = True
            if batch:
                acts.append(("cpb", batch))
            if not progress:
                raise CaptureError("the parties' tapes do not pair up (a receive no party "
                                   "sends)")
        if pending:
            raise CaptureError(f"{len(pending)} messages sent but never received")
        return acts

    def _free_party_graphs(self):
        from moose_amd.ops import native as nat

        torch.cuda.synchronize()
        for g, ex in self._party_graphs or []:
            nat.lib().mx_graph_free(g, ex)
        self._party_graphs = None

    def __del__(self):
        ex = getattr(self, "_launchers", None)
        if ex is not None:
            ex.shutdown(wait=False)
        hs = list(getattr(self, "_party_graphs", None) or [])
        hs += list(getattr(self, "_graph_handles", None) or [])
        for g, ex in hs:
            try:
                from moose_amd.ops import native as nat

                nat.lib().mx_graph_free(g, ex)
            except Exception:  # noqa: BLE001 - interpreter shutdown
                pass

    def _copy_stream(self, dev):
        s = self._copy_streams.get(dev)
        if s is None:
            s = self._copy_streams[dev] = torch.cuda.Stream(dev)
        return s

    def _schedule(self):
        from moose_amd.parallel.transport import CommStep
        from moose_amd.runtime.graphs import CaptureError

        n = len(self.tapes)
        steps = [t.steps for t in self.tapes]
        ptr, sent_done = [0] * n, [False] * n
        sent, recvd, pending = {}, {}, {}
        actions = []
        while any(ptr[p] < len(steps[p]) for p in range(n)):
            progress = False
            for p in range(n):
                while ptr[p] < len(steps[p]):
                    s = steps[p][ptr[p]]
                    if not isinstance(s, CommStep):
                        actions.append(("g", p, s))
                        ptr[p] += 1
                        progress = True
                        continue
                    if not sent_done[p]:
                        for t, dst in s.sends:
                            k = sent.get((p, dst), 0)
                            sent[(p, dst)] = k + 1
                            ev = torch.cuda.Event()
                            pending[(p, dst, k)] = (t, ev)
                            actions.append(("rec", p, ev))
                        sent_done[p] = True
                        progress = True
                    ready = {}
                    for _, src in s.recvs:
                        ready[src] = ready.get(src, 0) + 1
                    if any(sent.get((src, p), 0) < recvd.get((src, p), 0) + c
                           for src, c in ready.items()):
                        break  # a sender has not reached this message yet
                    for buf, src in s.recvs:
                        k = recvd.get((src, p), 0)
                        recvd[(src, p)] = k + 1
                        t, ev = pending.pop((src, p, k))
                        if t.numel() != buf.numel() or t.dtype != buf.dtype:
                            raise CaptureError(f"message {k} from party {src} to {p}: "
                                               f"{tuple(t.shape)} {t.dtype} sent, "
                                               f"{tuple(buf.shape)} {buf.dtype} expected")
                        actions.append(("cp", p, src, t.reshape(buf.shape), buf, ev))
                    ptr[p] += 1
                    sent_done[p] = False
                    progress = True
            if not progress:
                raise CaptureError("the parties' tapes do not pair up (a receive no party "
                                   "sends)")
        if pending:
            raise CaptureError(f"{len(pending)} messages sent but never received")
        return actions

    def replay(self, arguments: dict) -> Dict[str, dict]:
        import time

        if self._party_graphs is not None:
            from moose_amd.parallel.transport import TransportError

            try:
                return self._replay_streams(arguments)
            except TransportError as e:
                # a message never arrived (peer writes refused, a flag lost): this replay is
                # void -- redo it, and every later one, with the per-action replay
                import warnings

                warnings.warn(f"per-party stream graphs disabled: {e}", RuntimeWarning,
                              stacklevel=2)
                self._free_party_graphs()
                for err in self._errs:
                    err.zero_()
        if self._composed is not None:
            return self._replay_composed(arguments)
        return self._replay_actions(arguments)

    def _replay_actions(self, arguments: dict) -> Dict[str, dict]:
        """The per-action replay: one host thread issues every party's segments and the
        message copies, interleaved, on the parties' streams (event edges only)."""
        import time

        n = len(self.tapes)
        prev_dev = torch.cuda.current_device()
        prev = [torch.cuda.current_stream(d) for d in set(self.devices)]
        t0 = time.perf_counter()
        try:
            for p, tape in enumerate(self.tapes):
                s = self.streams[p]
                torch.cuda.set_stream(s)
                if self._ends is not None:  # the landing buffers are free again
                    for q in range(n):
                        if q != p:
                            s.wait_event(self._ends[q])
                tape.copy_arguments(arguments)
                tape._fill_keys()
            if self.shared_static:  # shared argument buffers: every upload before any reader
                evs = []
                for p in range(n):
                    e = torch.cuda.Event()
                    e.record(self.streams[p])
                    evs.append(e)
                for p in range(n):
                    for q in range(n):
                        if q != p:
                            self.streams[p].wait_event(evs[q])
            cur = -1
            for a in self.actions:
                p = a[1]
                if a[0] == "g":
                    if p != cur:
                        torch.cuda.set_stream(self.streams[p])
                        cur = p
                    a[2].replay()
                elif a[0] == "rec":
                    a[2].record(self.streams[p])
                else:
                    _, p, src, t, buf, ev = a
                    if self.devices[src] != self.devices[p]:
                        c = self._copy_stream(self.devices[src])
                        c.wait_event(ev)
                        torch.cuda.set_stream(c)  # the peer copy runs on the source GPU
                        torch.cuda.set_stream(self.streams[p])
                    else:
                        if p != cur:
                            torch.cuda.set_stream(self.streams[p])
                        self.streams[p].wait_event(ev)
                    cur = p
                    buf.copy_(t)
            ends = []
            for p in range(n):
                e = torch.cuda.Event()
                e.record(self.streams[p])
                ends.append(e)
            self._ends = ends
            self.issue_s.append(time.perf_counter() - t0)
            out = {}
            for p, tape in enumerate(self.tapes):
                torch.cuda.set_stream(self.streams[p])
                out[self.identities[p]] = tape._decode(tape.interp, tape.sess, tape.outs)
                tape.replays += 1
        finally:
            for s in prev:
                torch.cuda.set_stream(s)
            torch.cuda.set_device(prev_dev)
        return out

    def _replay_composed(self, arguments: dict) -> Dict[str, dict]:
        """One launch of the composed graph on the first party's stream, after every
        party's arguments and fresh keys were written on that same stream."""
        import time

        from moose_amd.ops import native as nat

        s = self.streams[0]
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            upload = not getattr(self, "_uploads_in_graph", False)
            for tape in self.tapes:
                tape.copy_arguments(arguments, upload=upload)
            t1 = time.perf_counter()
            in_graph = getattr(self, "_keys_in_graph", ())
            for p, tape in enumerate(self.tapes):
                if p not in in_graph:
                    tape._fill_keys()
            t2 = time.perf_counter()
            for ex in self._composed:
                nat.check(nat.lib().mx_graph_launch(ex, s.cuda_stream), "graph launch")
            t3 = time.perf_counter()
            self.issue_s.append(t3 - t0)
            # host time per replay: arguments staged, keys refreshed, graph launched
            self.issue_parts.append((t1 - t0, t2 - t1, t3 - t2))
            out = {}
            for p, tape in enumerate(self.tapes):
                out[self.identities[p]] = tape._decode(tape.interp, tape.sess, tape.outs)
                tape.replays += 1
        return out
