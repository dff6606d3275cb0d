"""Independent operations of different kinds sharing their message rounds (per-party sessions).

The reference's asynchronous session runs every operation as its own task, so independent
protocols advance side by side and a receive never blocks unrelated work
(``/root/reference/moose/src/execution/asynchronous.rs:456-530``).  Here a party runs its
operations from one interpreter loop; ``Interpreter._merge_unary`` and ``_batch_dots``
already fuse independent operations of ONE kind into one protocol run.  Different kinds --
a comparison beside an exponential, a division beside a sigmoid -- are run by
:class:`Lockstep` as coroutines on helper threads of the party:

* exactly one of them runs at a time, in a fixed order (no interleaving of kernel launches,
  no shared-scratch races), until it reaches a message round, where it parks;
* when every one of them has parked or finished, their rounds go out as ONE grouped
  exchange (the union of their sends and receives, in coroutine order), then each resumes;
* every operation draws its PRF nonces from its own scope (runtime/session.py
  nonce_scope), so the shares are bitwise those of running the operations one by one.

Every party forms the same groups (the interpreter groups by program structure) and runs the
same schedule, so the k-th message between two parties is still the k-th receive.  The
k coroutines cost the rounds of the longest instead of the sum of all (``stats.rounds``
counts the longest; bytes and messages are summed).  Works in eager evaluations and inside
tape captures (parallel/spmd_graphs.py): the merged round is one CommStep.
"""
from __future__ import annotations

import threading
from typing import Callable
from typing import List

import torch

from moose_amd.runtime.session import nonce_scope
from moose_amd.utils.telemetry import SessionStats

_TLS = threading.local()


def current(sess):
    """(lockstep, coroutine index) when the calling thread is a coroutine of a group running
    on ``sess``, else None."""
    w = getattr(_TLS, "worker", None)
    return w if w is not None and w[0].sess is sess else None


class _TransportProxy:
    """The session's transport while a group runs.  A coroutine parks at the points EVERY
    member of the placement reaches alike -- ``SPMDSession.party_exchange`` (through
    :func:`current`, also when this party has nothing to send or receive there) and the ring
    shift of a reshare -- so the parties' schedules stay identical.  Every other transport
    call (point-to-point moves, role-dependent grouped exchanges, key setup) runs at once,
    in that same deterministic order on every party, but on the scheduler's thread: a taped
    evaluation ends and restarts its capture segment at each message, and a thread-local
    hipGraph capture may only be ended by the thread that began it."""

    def __init__(self, ls: "Lockstep", real):
        self._ls, self._real = ls, real

    def __getattr__(self, name):
        attr = getattr(self._real, name)
        w = getattr(_TLS, "worker", None)
        if not callable(attr) or w is None or w[0] is not self._ls:
            return attr
        return lambda *a, **kw: self._ls.delegate(w[1], attr, a, kw)

    def shift(self, data, to_r, from_r):
        w = getattr(_TLS, "worker", None)
        if w is None or w[0] is not self._ls:
            return self._real.shift(data, to_r, from_r)
        data = data.contiguous()
        out = torch.empty_like(data)
        self._ls.park(w[1], [(data, to_r)], [(out, from_r)])
        return out


class _StatsProxy:
    """``sess.stats`` while a group runs: each coroutine records into its own SessionStats."""

    def __init__(self, ls: "Lockstep", real):
        self._ls, self._real = ls, real

    def _target(self):
        w = getattr(_TLS, "worker", None)
        return self._ls.stats[w[1]] if w is not None and w[0] is self._ls else self._real

    def __getattr__(self, name):
        return getattr(self._target(), name)


class Lockstep:
    """Run ``fns`` (independent operations of one party) as coroutines whose message rounds
    are merged (module doc).  ``scopes``: each coroutine's nonce scope."""

    def __init__(self, sess):
        self.sess = sess

    def park(self, k, sends, recvs):
        """Called on coroutine k's thread: hand its round to the scheduler and wait until
        the merged round has run."""
        self.pending[k] = (sends, recvs)
        self.back.release()
        self.go[k].acquire()
        if self.abort is not None:
            raise self.abort

    def delegate(self, k, fn, args, kwargs):
        """Called on coroutine k's thread: run ``fn`` on the scheduler's thread now (no
        park: the coroutine continues right after) and return its result."""
        self.calls[k] = (fn, args, kwargs)
        self.back.release()
        self.go[k].acquire()
        if self.abort is not None:
            raise self.abort
        res, err = self.replies.pop(k)
        if err is not None:
            raise err
        return res

    def _resume(self, k):
        """Run coroutine k until it parks or ends, serving its delegated calls."""
        self.go[k].release()
        while True:
            self.back.acquire()
            call = self.calls.pop(k, None)
            if call is None:
                return
            fn, args, kwargs = call
            try:
                self.replies[k] = (fn(*args, **kwargs), None)
            except BaseException as e:  # noqa: BLE001 - raised on the coroutine's thread
                self.replies[k] = (None, e)
            self.go[k].release()

    def run(self, fns: List[Callable], scopes: List[int]):
        n = len(fns)
        sess = self.sess
        self.go = [threading.Semaphore(0) for _ in range(n)]
        self.back = threading.Semaphore(0)
        self.pending, self.calls, self.replies = {}, {}, {}
        self.abort = None
        self.stats = [SessionStats() for _ in range(n)]
        results, errors, done = [None] * n, [None] * n, [False] * n
        cuda = sess.device.type == "cuda"
        stream = torch.cuda.current_stream(sess.device) if cuda else None

        def body(k):
            _TLS.worker = (self, k)
            try:
                if cuda:
                    torch.cuda.set_device(sess.device)
                    torch.cuda.set_stream(stream)
                self.go[k].acquire()
                if self.abort is None:
                    with nonce_scope(scopes[k]):
                        results[k] = fns[k]()
            except BaseException as e:  # noqa: BLE001 - re-raised by the scheduler
                errors[k] = e
            finally:
                done[k] = True
                _TLS.worker = None
                self.back.release()

        real_tr, real_stats = sess.tr, sess.stats
        sess.tr = _TransportProxy(self, real_tr)
        sess.stats = _StatsProxy(self, real_stats)
        threads = [threading.Thread(target=body, args=(k,), daemon=True,
                                    name=f"moose-lockstep-{k}") for k in range(n)]
        for t in threads:
            t.start()
        try:
            active = list(range(n))
            while active:
                for k in list(active):
                    self._resume(k)
                    if done[k]:
                        active.remove(k)
                if any(e is not None for e in errors):
                    break
                posts = [(k, self.pending.pop(k)) for k in sorted(self.pending)]
                if posts:  # ONE grouped round for every parked coroutine
                    real_tr.exchange([s for _, (ss, _) in posts for s in ss],
                                     [r for _, (_, rr) in posts for r in rr])
        except BaseException as e:  # noqa: BLE001 - release the parked coroutines
            self.abort = e
            raise
        finally:
            if self.abort is None and any(e is not None for e in errors):
                self.abort = next(e for e in errors if e is not None)
            for k in range(n):  # wake whatever still waits (an error ends the group)
                if not done[k]:
                    self.go[k].release()
            for t in threads:
                t.join(timeout=60)
            sess.tr, sess.stats = real_tr, real_stats
            for st in self.stats:  # bytes and messages add up; rounds run side by side
                for key, v in st.bytes.items():
                    real_stats.bytes[key] += v
                for key, v in st.messages.items():
                    real_stats.messages[key] += v
                real_stats.round_bytes += st.round_bytes
            real_stats.rounds += max((st.rounds for st in self.stats), default=0)
        if self.abort is not None:
            raise self.abort
        return results
