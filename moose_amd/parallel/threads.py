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

import queue
import threading
from typing import List
from typing import Optional

import torch

from moose_amd.ops import ring as R
from moose_amd.parallel.transport import TransportError


class Hub:
    """The mailboxes of one evaluation's parties (ordered pairs), plus failure state."""

    def __init__(self, devices: List, timeout: Optional[float] = None):
        self.devices = [torch.device(d) for d in devices]
        n = len(self.devices)
        self.boxes = {(s, d): queue.Queue() for s in range(n) for d in range(n) if s != d}
        self.failed: Optional[str] = None
        self.timeout = timeout
        self.lock = threading.Lock()

    def fail(self, why: str):
        with self.lock:
            if self.failed is None:
                self.failed = why


class ThreadTransport:
    """Transport API of :class:`~moose_amd.parallel.transport.Transport` (send / recv /
    shift / exchange) between the threads of a :class:`Hub`."""

    plans = False  # no headers: the values themselves travel
    tape = None
    stage = False

    def __init__(self, rank: int, hub: Hub):
        self.rank, self.hub = rank, hub
        self.world = len(hub.devices)
        self.device = hub.devices[rank]
        self.bytes_sent = 0
        self.messages = 0

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
        waited = 0.0
        while True:
            try:
                return box.get(timeout=0.05)
            except queue.Empty:
                waited += 0.05
                if self.hub.failed is not None:
                    raise TransportError(f"rank {self.rank}: no message from rank {src}: "
                                         f"session failed ({self.hub.failed})") from None
                if self.hub.timeout is not None and waited >= self.hub.timeout:
                    self.hub.fail(f"rank {self.rank} timed out waiting for rank {src}")
                    raise TransportError(f"rank {self.rank}: no message from rank {src} "
                                         f"within {self.hub.timeout} s") from None

    # -- typed values ------------------------------------------------------------------
    def send(self, v, dst: int):
        if isinstance(v, R.RT):
            y, ev = self._ship(v.data, dst)
            self._put(dst, ("rt", (y, v.bits), ev))
        elif isinstance(v, torch.Tensor):
            y, ev = self._ship(v, dst)
            self._put(dst, ("t", y, ev))
        else:  # host values (ints, floats, bytes, shapes, None) travel as they are
            self._put(dst, ("v", v, None))

    def recv(self, src: int, device=None):
        kind, val, ev = self._get(src)
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
        self.send(t, to_rank)
        return self.recv(from_rank)

    def exchange(self, sends, recvs):
        """Sends first (they never block), then each receive lands in its buffer."""
        for t, dst in sends:
            if t.numel():
                self.send(t, dst)
        for out, src in recvs:
            if out.numel():
                out.copy_(self.recv(src).reshape(out.shape))

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


def run_parties(comp, arguments: dict, identities: List[str], devices: List, storage: dict,
                fixedpoint_ring: int = 128, seed: Optional[int] = None,
                timeout: Optional[float] = None):
    """Evaluate ``comp`` with party ``identities[i]`` as a thread on ``devices[i]``.
    Returns ``(outputs, stats_by_identity, elapsed_us_by_identity)``; the outputs of every
    party merged (each output tag is materialised by the party that owns it)."""
    import time

    from moose_amd.compiler.passes import is_lowered
    from moose_amd.parallel.spmd import SPMDSession
    from moose_amd.runtime.interpreter import Interpreter

    hub = Hub(devices, timeout=timeout)
    role_ranks = {r: i for i, r in enumerate(identities)}
    results, stats, elapsed, errors = {}, {}, {}, {}
    lowered = is_lowered(comp)

    def party(i):
        ident, dev = identities[i], hub.devices[i]
        tr = ThreadTransport(i, hub)
        try:
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
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            elapsed[ident] = int((time.perf_counter() - t0) * 1e6)
            results[ident], stats[ident] = out, st
        except BaseException as e:  # noqa: BLE001 - reported after every party stopped
            errors[ident] = e
            hub.fail(f"{ident}: {type(e).__name__}: {e}")

    threads = [threading.Thread(target=party, args=(i,), name=f"moose-party-{identities[i]}",
                                daemon=True) for i in range(len(identities))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        # the first party to fail is the cause; the others saw TransportError because of it
        first = next((e for e in errors.values() if not isinstance(e, TransportError)),
                     next(iter(errors.values())))
        raise first
    merged = {}
    for ident in identities:
        merged.update(results[ident])
    return merged, stats, elapsed
