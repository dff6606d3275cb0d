"""Intra-party dataflow concurrency on the GPU: independent operations of a computation
run on different HIP streams ("lanes").

The reference executes every operation as its own async task, so independent operations
overlap (moose/src/execution/asynchronous.rs:456-530).  The MI355X counterpart keeps one
Python driver (launches are cheap and ordered) but gives the device the freedom the
reference's scheduler has: the toposorted operations are partitioned into chains, each
chain issues on its own stream, and only true data dependencies between chains become
event waits.  Under hipGraph capture the same waits become graph edges, so a replayed
evaluation executes independent branches concurrently on the CUs.

Plan (:class:`LanePlan`, host-only, unit tested on CPU): walk the ops in topological order;
an op continues the lane of a producer whose lane it would extend (that producer is the
lane's current tail), otherwise it starts on the next lane round-robin.  Every value read on
a lane other than its producer's gets one event (recorded after the producer) that the
consuming lane waits on once.

Runner (:class:`LaneRunner`): switches the current stream per op (every native launch and
ATen op picks it up via ``torch.cuda.current_stream``), inserts the waits, and marks
tensors read across lanes with ``record_stream`` so the caching allocator does not recycle
them under a still-running consumer.  ``fork``/``join`` bracket hipGraph capture segments:
every lane joins the capture by waiting on the main stream and is joined back into it
before the segment's capture ends.

Measured (profiles/r2_lanes_bench.jsonl, 8 independent secret sigmoid(x.w) branches): with
hipGraph replay 2 lanes cut 5.83 -> 4.92 ms at 4000 rows and 16.2 -> 14.5 ms at 40000 rows;
4 lanes add more barrier nodes than they win; eager evaluation is host-bound, so lanes only
add event overhead there.  Lanes are therefore opt-in (``MOOSEX_LANES`` / ``lanes=``).

Caches that hand one device tensor to many operations (public scalar constants, weight
vectors; ops/ring.py) and the key table (runtime/keys.py) drain the producing stream when
they publish a new buffer while lanes are active, so no lane reads a buffer another
stream is still producing.
"""
from __future__ import annotations

import os
from typing import Dict
from typing import List
from typing import Optional

import torch

ACTIVE = False  # a LaneRunner is driving the current evaluation (read by keys.py)
_TRACE = os.environ.get("MOOSEX_LANES_TRACE") == "1"


def _trace(*a):
    if _TRACE:
        print("[lanes]", *a, flush=True)


def default_lanes() -> int:
    return max(1, int(os.environ.get("MOOSEX_LANES", "1")))


class LanePlan:
    """Static chain decomposition of a toposorted op list onto ``nlanes`` lanes."""

    def __init__(self, ops, nlanes: int):
        self.nlanes = max(1, int(nlanes))
        self.lane: Dict[str, int] = {}
        self.consumers: Dict[str, List[str]] = {}
        tail: List[Optional[str]] = [None] * self.nlanes
        nxt = 0
        for op in ops:
            deps = [i for i in op.inputs if i in self.lane]
            for d in deps:
                self.consumers.setdefault(d, []).append(op.name)
            choice = None
            for d in deps:  # extend a chain whose tail is one of our producers
                ln = self.lane[d]
                if tail[ln] == d:
                    choice = ln
                    break
            if choice is None:
                choice = nxt
                nxt = (nxt + 1) % self.nlanes
            self.lane[op.name] = choice
            tail[choice] = op.name

    def crosses(self, name: str, lane: int) -> bool:
        """Some consumer of ``name`` (produced on ``lane``) runs on another lane."""
        return any(self.lane.get(c, lane) != lane for c in self.consumers.get(name, ()))

    def width(self) -> int:
        return len(set(self.lane.values()))


def tensors_of(v, out=None, depth=0):
    """Device tensors reachable from an interpreter value (LV / RepFixed / RepTensor / PV /
    HV / RT / containers)."""
    if out is None:
        out = {}
    if depth > 8 or v is None:
        return out
    if isinstance(v, torch.Tensor):
        if v.is_cuda:
            out[id(v)] = v
        return out
    if isinstance(v, (list, tuple)):
        for x in v:
            tensors_of(x, out, depth + 1)
        return out
    if isinstance(v, dict):
        for x in v.values():
            tensors_of(x, out, depth + 1)
        return out
    if isinstance(v, (str, bytes, int, float, bool)):
        return out
    slots = getattr(type(v), "__slots__", None)
    names = list(slots) if slots else list(getattr(v, "__dict__", {}).keys())
    for n in names:
        x = getattr(v, n, None)
        if x is not None and not callable(x):
            tensors_of(x, out, depth + 1)
    return out


class LaneRunner:
    """Drives one evaluation's lanes (see module docstring)."""

    def __init__(self, device, nlanes: int):
        self.device = torch.device(device)
        self.nlanes = max(1, int(nlanes))
        self.streams = None
        self.plan: Optional[LanePlan] = None

    # -- evaluation bracket -----------------------------------------------------------
    def start(self, ops):
        global ACTIVE
        self.main = torch.cuda.current_stream(self.device)
        if self.streams is None:
            self.streams = [None] + [torch.cuda.Stream(self.device)
                                     for _ in range(self.nlanes - 1)]
        self.streams[0] = self.main
        self.plan = LanePlan(ops, self.nlanes)
        # every event of this evaluation stays alive until the next one starts: HIP keeps
        # references to events recorded during a stream capture until the capture ends
        self._keep = []
        self.where: Dict[str, int] = {}  # value -> lane it was produced on
        self.events: Dict[str, torch.cuda.Event] = {}
        self.waited = [set() for _ in range(self.nlanes)]
        self.used = [False] * self.nlanes
        self.cur = 0
        self.fork()
        ACTIVE = True

    def finish(self):
        global ACTIVE
        try:
            self.join()
        finally:
            torch.cuda.set_stream(self.main)
            ACTIVE = False

    # -- capture segments ----------------------------------------------------------------
    def fork(self):
        """Lanes start after everything issued on the main stream so far (a hipGraph
        capture segment's start).  A lane waits on this point when it is first used, so
        every stream that joins a capture does work in it and is joined back by join()
        (a stream left joined but unjoined breaks the capture)."""
        torch.cuda.set_stream(self.main)
        self.fork_ev = self._event()
        self.fork_ev.record(self.main)
        _trace("fork", "capturing" if torch.cuda.is_current_stream_capturing() else "")
        self.used = [False] * self.nlanes
        self.seg = getattr(self, "seg", 0) + 1
        # everything produced before is ordered before every lane now (and events of an
        # ended capture segment must not be waited on in the next one)
        self.events = {}
        self.waited = [set() for _ in range(self.nlanes)]

    def join(self):
        """The main stream waits on every lane used since the last fork."""
        torch.cuda.set_stream(self.main)
        for ln in range(1, self.nlanes):
            if self.used[ln]:
                ev = self._event()
                ev.record(self.streams[ln])
                self.main.wait_event(ev)
                _trace("join lane", ln)
        self.used = [False] * self.nlanes

    # -- per operation -------------------------------------------------------------------
    def enter(self, op, env):
        ln = self.plan.lane.get(op.name, 0)
        s = self.streams[ln]
        if ln and not self.used[ln]:
            s.wait_event(self.fork_ev)
            _trace("lane", ln, "waits fork")
        for d in op.inputs:
            src = self.where.get(d, ln)
            if src == ln:
                continue
            ev = self.events.get(d)
            if ev is not None and d not in self.waited[ln]:
                s.wait_event(ev)
                self.waited[ln].add(d)
                _trace("lane", ln, "waits", d, "from lane", src)
            for t in tensors_of(env.get(d)).values():
                t.record_stream(s)
        self.cur = ln
        self.used[ln] = True
        _trace("enter", op.name, op.kind, "lane", ln)
        torch.cuda.set_stream(s)

    def ordered_here(self, names) -> bool:
        """Every value in ``names`` is safe to read on the current lane without a new wait:
        produced on it, produced before the lanes forked, or already waited on (its tensors
        then carry a record_stream for this lane).  Ops executed ahead of their own turn
        (batched Dots) are restricted to such operands."""
        ln = self.cur
        return all(self.where.get(n, ln) == ln or n in self.waited[ln] for n in names)

    def leave(self, names):
        """Values ``names`` were just produced on the current lane."""
        ln = self.cur
        ev = None
        for n in names:
            self.where[n] = ln
            if self.plan.crosses(n, ln):
                if ev is None:
                    ev = self._event()
                    ev.record(self.streams[ln])
                self.events[n] = ev
                _trace("event for", n, "on lane", ln)
        torch.cuda.set_stream(self.main)

    def mark(self):
        """A point on the current stream (values produced outside an op's own output,
        e.g. conversions memoised for a later op); see wait_mark."""
        st = torch.cuda.current_stream(self.device)
        ev = self._event()
        ev.record(st)
        return ev, self.seg, st.cuda_stream

    def _event(self):
        ev = torch.cuda.Event()
        self._keep.append(ev)
        return ev

    def wait_mark(self, mark, value):
        """The current stream waits on ``mark`` (unless a fork since has ordered it) and
        keeps ``value``'s tensors alive for it."""
        ev, seg, origin = mark
        s = torch.cuda.current_stream(self.device)
        # same stream: already ordered (and a capture must not wait on its own stream's
        # event: HIP's stream capture crashes at EndCapture on such a side-stream self-wait)
        if seg == self.seg and s.cuda_stream != origin:
            s.wait_event(ev)
        for t in tensors_of(value).values():
            t.record_stream(s)
