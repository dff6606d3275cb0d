"""Tracing, counters and per-session metrics.

* :class:`SessionStats` -- bytes sent per (sender, receiver) pair, communication rounds,
  elapsed time per role (the reference only reports per-role ``elapsed_time``,
  ``choreography/grpc.rs:150,187-192``).
* :func:`span` -- a context manager recording a Chrome-trace event and, on GPU, a roctx
  range (``torch.cuda.nvtx`` maps to roctx on ROCm) so protocol steps show up in
  ``rocprofv3 --marker-trace`` timelines.
* ``MOOSEX_TRACE=path.json`` dumps all spans at exit; ``MOOSEX_LOG`` sets the log level.
"""
from __future__ import annotations

import atexit
import json
import logging
import os
import threading
import time
from collections import defaultdict
from contextlib import contextmanager
from contextlib import nullcontext

_LOG = logging.getLogger("moose_amd")
if os.environ.get("MOOSEX_LOG"):
    logging.basicConfig(level=os.environ["MOOSEX_LOG"].upper())


def get_logger():
    return _LOG


class SessionStats:
    def __init__(self):
        self.bytes = defaultdict(int)
        self.messages = defaultdict(int)
        self.rounds = 0
        self.round_bytes = 0
        self.elapsed = {}

    def record_send(self, src, dst, nbytes, count=1):
        self.bytes[(src, dst)] += int(nbytes) * count
        self.messages[(src, dst)] += count

    def record_round(self, nbytes, count=1):
        self.rounds += count
        self.round_bytes += int(nbytes) * count

    def as_dict(self):
        return {
            "rounds": self.rounds,
            "reshare_bytes": self.round_bytes,
            "bytes": {f"{a}->{b}": v for (a, b), v in self.bytes.items()},
            "messages": {f"{a}->{b}": v for (a, b), v in self.messages.items()},
            "elapsed_us": dict(self.elapsed),
        }


_EVENTS = []
_EV_LOCK = threading.Lock()
_TRACE_PATH = os.environ.get("MOOSEX_TRACE")


def _nvtx():
    try:
        import torch

        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:  # pragma: no cover
        pass
    return None


_ROCTX = os.environ.get("MOOSEX_ROCTX")
_NULL_SPAN = nullcontext()


def span(name, **args):
    """Record a named interval (Chrome trace + roctx range when on GPU).  A shared no-op
    context when neither tracing nor roctx ranges are on (spans sit on every protocol
    call)."""
    if not _TRACE_PATH and not _ROCTX:
        return _NULL_SPAN
    return _span(name, **args)


@contextmanager
def _span(name, **args):
    nv = _nvtx()
    if nv is not None:
        nv.range_push(name)
    t0 = time.perf_counter_ns()
    try:
        yield
    finally:
        t1 = time.perf_counter_ns()
        if nv is not None:
            nv.range_pop()
        if _TRACE_PATH:
            with _EV_LOCK:
                _EVENTS.append(
                    {
                        "name": name,
                        "ph": "X",
                        "ts": t0 / 1e3,
                        "dur": (t1 - t0) / 1e3,
                        "pid": os.getpid(),
                        "tid": threading.get_ident() % 100000,
                        "args": args,
                    }
                )


def enable_tracing(path: str):
    """Turn span recording on at run time (CLI ``--telemetry``); dumped at exit.  The
    reference exports spans to Jaeger (``reindeer.rs:6-30``); here a Chrome trace."""
    global _TRACE_PATH
    first = _TRACE_PATH is None
    _TRACE_PATH = path
    if first:
        atexit.register(dump_trace)


def dump_trace(path=None):
    path = path or _TRACE_PATH
    if not path:
        return
    with _EV_LOCK:
        evs = list(_EVENTS)
    with open(path, "w") as f:
        json.dump({"traceEvents": evs}, f)


if _TRACE_PATH:
    atexit.register(dump_trace)
