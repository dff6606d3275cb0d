"""Fail-loudly machinery for multi-rank benchmark runs (``bench.py``).

A multi-GPU run that hangs (a rank stuck in an RCCL exchange, a dead peer, a wiring bug)
must end with a diagnosable record, not a silent timeout.  Three pieces:

* :class:`Progress` -- every rank records the phase it is in (``init``, ``preflight``,
  ``warmup``, ``timed``, ...) in a small file of a per-run directory.  A watchdog thread
  re-armed at each phase fires when a phase overruns its budget: rank 0 prints the run's
  JSON line -- the finished result with the failure recorded in it when the headline metric
  was already measured, else an ``"error"`` line naming the stalled ranks and every rank's
  phase -- and every rank exits (status 0 when the headline was complete, 3 otherwise).
* :func:`supervise` -- the parent of a self-launched ``--gpus N`` run (which never touches
  the GPU) waits for the rank group with a wall-clock limit, kills the whole process group
  on expiry and prints the same error line from the ranks' phase files.
* :func:`stall_if_requested` -- test hook: ``MOOSEX_BENCH_STALL=<rank>:<phase>`` makes that
  rank hang at the start of that phase (used by the CPU test of the watchdog).

Reference: the reference's client collects per-worker elapsed times and fails the run when a
worker errors (``moose/src/execution/grpc.rs:105-145``); its networking retries sends with
backoff (``networking/grpc.rs:106-134``).  Here failure is bounded by phase budgets.
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import threading
import time
from typing import Callable
from typing import Dict
from typing import Optional


def run_dir(explicit: Optional[str] = None) -> str:
    """The per-run directory shared by all ranks of one node (same MASTER_PORT / run id)."""
    d = explicit or os.environ.get("MOOSEX_BENCH_RUN_DIR")
    if not d:
        # ranks of one launch share the launcher (their parent process) and its port
        tag = "{}_{}_{}".format(os.environ.get("TORCHELASTIC_RUN_ID", "solo"),
                                os.environ.get("MASTER_PORT", "0"), os.getppid())
        d = os.path.join("/tmp", f"moosex_bench_{tag}")
    os.makedirs(d, exist_ok=True)
    return d


def read_phases(d: str, world: int) -> Dict[int, dict]:
    out = {}
    for r in range(world):
        try:
            with open(os.path.join(d, f"rank{r}.json")) as f:
                out[r] = json.load(f)
        except (OSError, ValueError):
            out[r] = {"phase": "not started", "t": None}
    return out


def stalled_ranks(phases: Dict[int, dict]):
    """Ranks furthest behind -- earliest phase (by order of entry), then fewest steps
    entered in it: the ones the others wait for."""
    def pos(p):
        return (p.get("seq", -1), p.get("step", -1))
    if not phases:
        return []
    lo = min(pos(p) for p in phases.values())
    return sorted(r for r, p in phases.items() if pos(p) == lo)


def stall_if_requested(rank: int, phase: str):
    """Test hooks: ``MOOSEX_BENCH_STALL=rank:phase`` hangs that rank at the phase's entry,
    ``MOOSEX_BENCH_FAIL=rank:phase`` raises there."""
    for var in ("MOOSEX_BENCH_STALL", "MOOSEX_BENCH_FAIL"):
        spec = os.environ.get(var, "")
        if not spec:
            continue
        r, _, ph = spec.partition(":")
        if int(r) != rank or ph != phase:
            continue
        if var == "MOOSEX_BENCH_FAIL":
            raise RuntimeError(f"MOOSEX_BENCH_FAIL in {phase}")
        print(f"[bench] rank {rank}: MOOSEX_BENCH_STALL -> hanging in {phase}", file=sys.stderr,
              flush=True)
        while True:
            time.sleep(3600)


def failed_ranks(phases: Dict[int, dict]):
    """Ranks whose phase record says they raised (``Progress.fail``)."""
    return sorted(r for r, p in phases.items() if p.get("failed"))


class Progress:
    """Per-rank phase record + watchdog (module doc)."""

    def __init__(self, rank: int, world: int, budget_s: float, base_line: Callable[[], dict],
                 directory: Optional[str] = None):
        self.rank, self.world = rank, world
        self.dir = run_dir(directory)
        self.base_line = base_line  # -> the JSON line so far (metric, config, ...)
        self.result: Optional[dict] = None  # the finished headline line, once measured
        self.seq = 0
        self.step = -1  # operations entered in the current phase (tick)
        self.phase_name = "init"
        self.deadline = time.monotonic() + budget_s
        self.t0 = time.monotonic()
        self._lock = threading.Lock()
        self._wlock = threading.Lock()
        self._fired = False
        self.failed: Optional[str] = None
        self._write()
        t = threading.Thread(target=self._watch, name="bench-watchdog", daemon=True)
        t.start()

    def phase(self, name: str, budget_s: float):
        with self._lock:
            self.seq += 1
            self.step = -1
            self.phase_name = name
            self.deadline = time.monotonic() + budget_s
        self._write()
        stall_if_requested(self.rank, name)

    def tick(self, k: int):
        """About to start operation ``k`` of the phase (a plain store: the watchdog
        thread publishes it, so this is free inside timed loops)."""
        self.step = k

    def headline_done(self, line: dict):
        self.result = line

    def disarm(self):
        with self._lock:
            self.deadline = float("inf")

    def _write(self):
        # the main thread (phase entry) and the watchdog thread (tick publication) both
        # write: one at a time, or one's rename finds the other's temp file gone
        with self._wlock:
            rec = {"phase": self.phase_name, "seq": self.seq, "step": self.step,
                   "pid": os.getpid(), "t": round(time.monotonic() - self.t0, 3)}
            if self.failed:
                rec["failed"] = self.failed
            self._written = (self.seq, self.step)
            tmp = os.path.join(self.dir, f".rank{self.rank}.tmp")
            try:
                with open(tmp, "w") as f:
                    json.dump(rec, f)
                os.replace(tmp, os.path.join(self.dir, f"rank{self.rank}.json"))
            except OSError as e:  # a phase record is diagnostics: never fail the run on it
                print(f"[bench] rank {self.rank}: phase record not written: {e}",
                      file=sys.stderr, flush=True)

    def _watch(self):
        n = 0
        while True:
            time.sleep(0.5)
            n += 1
            if (self.seq, self.step) != getattr(self, "_written", None):
                self._write()
            # a rank that raised ends the run now, not when this rank's phase budget runs
            # out (its peers would otherwise wait in a collective until then)
            bad = failed_ranks(read_phases(self.dir, self.world)) if n % 2 == 0 else []
            bad = [r for r in bad if r != self.rank]
            with self._lock:
                late = (time.monotonic() > self.deadline or bad) and not self._fired
                if late:
                    self._fired = True
            if late:
                self.fire(f"rank {bad[0]} failed" if bad else None)

    def fail(self, what: str):
        """An exception on this rank: report it like a stall (rank 0 prints the line),
        then let the caller re-raise."""
        with self._lock:
            if self._fired:
                return
            self._fired = True
        self.failed = f"{what} in phase {self.phase_name!r}"
        self._write()
        self.fire(f"rank {self.rank}: {self.failed}", exit=False)

    def fire(self, msg: Optional[str] = None, exit: bool = True):
        phases = read_phases(self.dir, self.world)
        msg = msg or (f"rank {self.rank}: phase {self.phase_name!r} exceeded its budget "
                      f"({time.monotonic() - self.t0:.1f} s into the run)")
        print(f"[bench] WATCHDOG {msg}; phases: {json.dumps(phases)}", file=sys.stderr,
              flush=True)
        code = 0 if self.result is not None else 3
        if self.rank == 0:
            if self.result is not None:  # the headline is measured: keep it, note the stall
                line = dict(self.result)
                line.setdefault("errors", []).append(
                    {"phase": self.phase_name, "stalled_ranks": stalled_ranks(phases),
                     "phases": phases})
            else:
                line = dict(self.base_line(), value=None, error=msg,
                            stalled_ranks=stalled_ranks(phases), phases=phases)
            print(json.dumps(line), flush=True)
        else:
            # let rank 0 print first: the launcher tears the group down when a rank exits
            time.sleep(5)
        sys.stdout.flush()
        sys.stderr.flush()
        if exit:
            os._exit(code)


def supervise(cmd, env, world: int, limit_s: float, base_line: dict, directory: str) -> int:
    """Run the rank launcher ``cmd`` in its own process group; on expiry of ``limit_s``
    kill the group and print an error JSON line built from the ranks' phase files."""
    p = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return p.wait(timeout=limit_s)
    except subprocess.TimeoutExpired:
        pass
    phases = read_phases(directory, world)
    for sig, grace in ((signal.SIGTERM, 10), (signal.SIGKILL, 5)):
        try:
            os.killpg(p.pid, sig)
        except ProcessLookupError:
            break
        try:
            p.wait(timeout=grace)
            break
        except subprocess.TimeoutExpired:
            continue
    line = dict(base_line, value=None,
                error=f"rank group did not finish within {limit_s:.0f} s (killed)",
                stalled_ranks=stalled_ranks(phases), phases=phases)
    print(json.dumps(line), flush=True)
    return 3
