"""Fail-loudly machinery for benchmark runs (``bench.py``): one wall-clock deadline, phase
budgets carved out of it, and a fallback ladder of fresh attempts.

A multi-GPU run that hangs (a rank stuck in an RCCL exchange, a dead peer, a wiring bug)
must still end -- well inside the driver's own limit -- with a JSON line: the measurement
if one was taken (possibly by a fallback configuration, labelled as such), else an error
naming the stalled ranks.  Pieces:

* :class:`Clock` -- the run's absolute deadline (``--deadline`` seconds from the start,
  default :data:`DEFAULT_DEADLINE_S`, under the driver's 600 s) and the time by which the
  current attempt must have measured its headline (earlier: the fallbacks' reserve).
* :class:`Progress` -- every rank records the phase it is in (``init``, ``rendezvous``,
  ``preflight``, ``warmup``, ``timed``, extras ...) in a small file of a per-attempt
  directory, and the seconds each phase took (``phase_s`` in the line).  A watchdog thread
  re-armed at each phase fires when a phase overruns its budget (its cap from
  :data:`PHASE_CAPS`, clipped to the time left).  An optional extra after the headline is
  skipped (and listed under ``skipped``) when less than its expected need is left.
* :func:`rank_supervisor` -- under a launcher (``torch.distributed.run``; every rank runs it)
  the rank processes never touch the GPU: each spawns its worker as a child process and
  the supervisors walk the ladder together, rank 0's deciding through small files in the
  shared run directory.  An attempt that fails or stalls before its headline is killed on
  every rank (fresh process, fresh port, fresh communicators -- never a re-exec) and the
  next rung starts: cyclic with 2 step streams -> 1 step stream -> stacked over gloo.
  Rank 0's supervisor prints the one JSON line, with ``attempts: [{layout, streams,
  backend, outcome, phase, ...}]``.
* :func:`supervise` -- the parent of a self-launched ``--gpus N`` run waits for the launcher
  with a wall-clock limit (the deadline plus a grace), kills its process group on expiry
  and prints an error line from the phase files.
* :func:`stall_if_requested` -- test hooks: ``MOOSEX_BENCH_STALL=<rank>:<phase>[:<attempt>]``
  makes that rank hang at the start of that phase of that attempt (default 0),
  ``MOOSEX_BENCH_FAIL`` makes it raise there.

This module is loaded by path from the supervising processes: standard library only (no
torch import, nothing that could touch the GPU).

Reference: the reference's client collects per-worker elapsed times and fails the run when a
worker errors (``moose/src/execution/grpc.rs:105-145``; its benchmark takes the max over
the workers, ``benchmarks/pymoose/dot_product.py:124-139``); its networking retries sends
with backoff (``networking/grpc.rs:106-134``).  Here failure is bounded by one deadline.
"""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import Callable
from typing import Dict
from typing import List
from typing import Optional

DEFAULT_DEADLINE_S = 540.0  # the driver kills a bench run at 600 s

# (cap, need) seconds per phase at the default deadline (scaled with --deadline).  The cap is
# the watchdog budget; an optional extra after the headline only starts when at least
# ``need`` seconds are left.  init + rendezvous share one 120 s cap (from the process start).
PHASE_CAPS = {
    "init": (120, 0), "rendezvous": (120, 0), "preflight": (60, 0), "warmup": (120, 0),
    "timed": (180, 0),
    "report": (30, 0), "check": (60, 10), "zero_slot": (60, 15), "link_probe": (60, 15),
    "lr": (120, 30), "lr_spmd": (120, 30), "spmd_configs": (180, 45), "done": (30, 0),
}
MARGIN_S = 3.0  # a phase ends this long before the deadline it is clipped to


def _now():
    return time.time()


class Clock:
    """Absolute (epoch) deadlines of one attempt: ``deadline_at`` for the whole run,
    ``headline_by`` for the headline measurement; ``scale`` = deadline length / 540 s."""

    def __init__(self, deadline_at: float, headline_by: Optional[float] = None,
                 scale: float = 1.0):
        self.deadline_at = deadline_at
        self.headline_by = min(headline_by or deadline_at, deadline_at)
        self.scale = scale

    @classmethod
    def starting_now(cls, deadline_s: float = DEFAULT_DEADLINE_S):
        return cls(_now() + deadline_s, None, deadline_s / DEFAULT_DEADLINE_S)

    @classmethod
    def from_env(cls, default_s: float = DEFAULT_DEADLINE_S):
        at = os.environ.get("MOOSEX_BENCH_DEADLINE_AT")
        if not at:
            return cls.starting_now(default_s)
        return cls(float(at), float(os.environ.get("MOOSEX_BENCH_HEADLINE_BY") or at),
                   float(os.environ.get("MOOSEX_BENCH_SCALE") or 1.0))

    def cap(self, phase: str) -> float:
        return PHASE_CAPS.get(phase, (60, 0))[0] * self.scale

    def need(self, phase: str) -> float:
        return PHASE_CAPS.get(phase, (60, 0))[1] * self.scale


def run_dir(explicit: Optional[str] = None) -> str:
    """The per-run directory shared by all ranks of one node (same launcher: same
    MASTER_PORT and parent process)."""
    d = explicit or os.environ.get("MOOSEX_BENCH_RUN_DIR")
    if not d:
        tag = "{}_{}_{}".format(os.environ.get("TORCHELASTIC_RUN_ID", "solo"),
                                os.environ.get("MASTER_PORT", "0"), os.getppid())
        d = os.path.join("/tmp", f"moosex_bench_{tag}")
    os.makedirs(d, exist_ok=True)
    return d


def _write_json(path: str, rec: dict):
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        json.dump(rec, f)
    os.replace(tmp, path)


def _read_json(path: str) -> Optional[dict]:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def read_phases(d: str, world: int) -> Dict[int, dict]:
    out = {}
    for r in range(world):
        out[r] = _read_json(os.path.join(d, f"rank{r}.json")) or {"phase": "not started",
                                                                  "t": None}
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
    """Test hooks: ``MOOSEX_BENCH_STALL=rank:phase[:attempt]`` hangs that rank at the phase's
    entry, ``MOOSEX_BENCH_FAIL=rank:phase[:attempt]`` raises there (attempt: default 0,
    ``*`` for every attempt)."""
    attempt = int(os.environ.get("MOOSEX_BENCH_ATTEMPT", "0"))
    for var in ("MOOSEX_BENCH_STALL", "MOOSEX_BENCH_FAIL"):
        spec = os.environ.get(var, "")
        if not spec:
            continue
        parts = spec.split(":")
        r, ph = int(parts[0]), parts[1]
        at = parts[2] if len(parts) > 2 else "0"  # "*": every attempt
        if r != rank or ph != phase or at not in ("*", str(attempt)):
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
    """Per-rank phase record + watchdog (module doc).

    ``result_path`` (a supervised worker, rank 0): the line is published there -- at the
    headline and again at every later phase entry -- instead of printed; the supervisor
    prints it."""

    def __init__(self, rank: int, world: int, clock: Clock, base_line: Callable[[], dict],
                 directory: Optional[str] = None, result_path: Optional[str] = None,
                 t0: Optional[float] = None):
        self.rank, self.world = rank, world
        self.clock = clock
        self.dir = run_dir(directory)
        self.base_line = base_line  # -> the JSON line so far (metric, config, ...)
        self.result_path = result_path if rank == 0 else None
        self.result: Optional[dict] = None  # the finished headline line, once measured
        self.seq = 0
        self.step = -1  # operations entered in the current phase (tick)
        self.phase_name = "init"
        self.t0 = time.monotonic() if t0 is None else t0  # the process start, if known
        self.phase_t0 = self.t0
        self.phase_s: Dict[str, float] = {}
        self.skipped: List[str] = []
        self.deadline = self._limit_mono(clock.cap("init"))
        self._lock = threading.Lock()
        self._wlock = threading.Lock()
        self._fired = False
        self.failed: Optional[str] = None
        self._write()
        t = threading.Thread(target=self._watch, name="bench-watchdog", daemon=True)
        t.start()

    # ----------------------------------------------------------------------- budgets
    def _limit_mono(self, cap: float) -> float:
        """Monotonic time at which a phase starting now with cap ``cap`` is overdue."""
        end = self.clock.deadline_at if self.result is not None else self.clock.headline_by
        left = end - _now() - MARGIN_S
        return time.monotonic() + max(1.0, min(cap, left))

    def remaining(self) -> float:
        return self.clock.deadline_at - _now()

    def phase(self, name: str, cap: Optional[float] = None):
        now = time.monotonic()
        if cap is None:
            cap = self.clock.cap(name)
        if name == "rendezvous":  # init + rendezvous share one cap
            cap = max(1.0, cap - (now - self.t0))
        with self._lock:
            self.phase_s[self.phase_name] = round(
                self.phase_s.get(self.phase_name, 0.0) + now - self.phase_t0, 3)
            self.phase_t0 = now
            self.seq += 1
            self.step = -1
            self.phase_name = name
            self.deadline = self._limit_mono(cap)
        self._write()
        self.publish()
        stall_if_requested(self.rank, name)

    def extra_fits(self, name: str) -> bool:
        """Whether the optional phase ``name`` (after the headline) has at least its expected
        need left before the deadline.  Ranks must agree on the answer (the caller reduces
        it over the group) before entering the phase or recording the skip."""
        return self.remaining() - MARGIN_S >= max(self.clock.need(name), 1.0)

    def skip(self, name: str):
        self.skipped.append(name)

    def tick(self, k: int):
        """About to start operation ``k`` of the phase (a plain store: the watchdog
        thread publishes it, so this is free inside timed loops)."""
        self.step = k

    # ------------------------------------------------------------------------ result
    def headline_done(self, line: dict):
        self.result = line
        self.publish()

    def final_line(self, line: Optional[dict] = None) -> dict:
        line = dict(line if line is not None else (self.result or {}))
        line.pop("phase_s", None)
        now = time.monotonic()
        ph = dict(self.phase_s)
        ph[self.phase_name] = round(ph.get(self.phase_name, 0.0) + now - self.phase_t0, 3)
        line["phase_s"] = ph
        if self.skipped:
            line["skipped"] = list(self.skipped)
        return line

    def publish(self, line: Optional[dict] = None, complete: bool = False):
        """Rank 0 of a supervised worker: write the line so far to the result file."""
        if self.result_path is None or (line is None and self.result is None):
            return
        rec = self.final_line(line)
        rec["complete"] = complete
        rec["phase_at_publish"] = self.phase_name
        try:
            _write_json(self.result_path, rec)
        except OSError as e:
            print(f"[bench] result not written: {e}", file=sys.stderr, flush=True)

    def emit(self, line: dict):
        """The finished line: printed (unsupervised) or published as complete."""
        if self.result_path is not None:
            self.publish(line, complete=True)
        elif self.rank == 0:
            print(json.dumps(self.final_line(line)), flush=True)

    def disarm(self):
        with self._lock:
            self.deadline = float("inf")

    # ---------------------------------------------------------------------- watchdog
    def _write(self):
        # the main thread (phase entry) and the watchdog thread (tick publication) both
        # write: one at a time, or one's rename finds the other's temp file gone
        with self._wlock:
            rec = {"phase": self.phase_name, "seq": self.seq, "step": self.step,
                   "pid": os.getpid(), "t": round(time.monotonic() - self.t0, 3),
                   "attempt": int(os.environ.get("MOOSEX_BENCH_ATTEMPT", "0"))}
            if self.failed:
                rec["failed"] = self.failed
            self._written = (self.seq, self.step)
            try:
                _write_json(os.path.join(self.dir, f"rank{self.rank}.json"), rec)
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
        """An exception on this rank: report it like a stall (rank 0 reports the line),
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
                line["errors"] = list(line.get("errors", [])) + [
                    {"phase": self.phase_name, "error": msg,
                     "stalled_ranks": stalled_ranks(phases), "phases": phases}]
            else:
                line = dict(self.base_line(), value=None, error=msg,
                            stalled_ranks=stalled_ranks(phases), phases=phases)
            self.emit(line)
        else:
            # let rank 0 report first: the launcher tears the group down when a rank exits
            time.sleep(5)
        sys.stdout.flush()
        sys.stderr.flush()
        if exit:
            os._exit(code)


# ------------------------------------------------------------------------------------------
# supervisors (standard library only: these processes never touch the GPU)
# ------------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _die_with_parent():
    """preexec_fn: the worker gets SIGKILL when its supervisor dies (a launcher that kills
    the supervisors must not leave workers holding the GPU)."""
    try:
        import ctypes

        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL)  # PR_SET_PDEATHSIG
    except Exception:  # noqa: BLE001 - best effort
        pass


def _kill(p: subprocess.Popen, grace: float = 5.0):
    if p is None or p.poll() is not None:
        return
    for sig in (signal.SIGTERM, signal.SIGKILL):
        try:
            p.send_signal(sig)
        except ProcessLookupError:
            return
        try:
            p.wait(timeout=grace)
            return
        except subprocess.TimeoutExpired:
            continue


def _spawn(script: str, argv: List[str], env: dict) -> subprocess.Popen:
    return subprocess.Popen([sys.executable, script] + list(argv), env=env,
                            preexec_fn=_die_with_parent)


def _worker_env(att: dict, rank_dir: str, rank: int) -> dict:
    env = dict(os.environ)
    env.update({"MASTER_PORT": str(att["port"]), "MASTER_ADDR": env.get("MASTER_ADDR",
                                                                        "127.0.0.1"),
                "TORCHELASTIC_USE_AGENT_STORE": "False",  # worker rank 0 hosts the store
                "MOOSEX_BENCH_CHILD": "1", "MOOSEX_BENCH_ATTEMPT": str(att["k"]),
                "MOOSEX_BENCH_RUN_DIR": rank_dir,
                "MOOSEX_BENCH_DEADLINE_AT": repr(att["deadline_at"]),
                "MOOSEX_BENCH_HEADLINE_BY": repr(att["headline_by"]),
                "MOOSEX_BENCH_SCALE": repr(att["scale"])})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if rank == 0:
        env["MOOSEX_BENCH_RESULT"] = os.path.join(rank_dir, "result.json")
    return env


def _install_term_handler(get_child):
    def handler(signum, frame):  # noqa: ARG001
        _kill(get_child(), grace=3.0)
        os._exit(128 + signum)
    signal.signal(signal.SIGTERM, handler)
    signal.signal(signal.SIGINT, handler)


def rank_supervisor(script: str, rank: int, world: int, ladder: List[dict],
                    deadline_s: float, base_line: dict, directory: Optional[str] = None,
                    poll_s: float = 0.25) -> int:
    """One per rank under a launcher (module doc).  ``ladder``: rungs ``{"argv": [...],
    "label": {...}, "reserve_s": s}`` -- ``reserve_s`` is what the rung needs at least
    (the earlier rungs' headline deadlines leave it free).  Returns the exit status."""
    t_start = _now()
    d = run_dir(directory)
    child = [None]
    _install_term_handler(lambda: child[0])
    if rank == 0:
        return _lead(script, world, ladder, deadline_s, base_line, d, t_start, child, poll_s)
    return _follow(script, rank, world, deadline_s, d, t_start, child, poll_s)


def _lead(script, world, ladder, deadline_s, base_line, d, t_start, child, poll_s):
    for name in os.listdir(d):  # a reused directory: nothing stale may steer this run
        if name.startswith(("attempt", "abort", "end", "exit", "reaped")):
            try:
                os.remove(os.path.join(d, name))
            except OSError:
                pass
    nonce = f"{os.getpid()}-{t_start:.6f}"
    deadline_at = t_start + deadline_s
    scale = deadline_s / DEFAULT_DEADLINE_S
    attempts, final, code = [], None, 3
    for k, rung in enumerate(ladder):
        reserve = sum(r["reserve_s"] for r in ladder[k + 1:]) * scale
        headline_by = deadline_at - reserve
        if headline_by - _now() < rung["reserve_s"] * scale * 0.5:
            attempts.append(dict(rung["label"], outcome="skipped (no time left)"))
            continue
        rdir = os.path.join(d, f"a{k}")
        os.makedirs(rdir, exist_ok=True)
        for name in os.listdir(rdir):
            try:
                os.remove(os.path.join(rdir, name))
            except OSError:
                pass
        att = {"k": k, "nonce": nonce, "port": _free_port(), "argv": rung["argv"],
               "dir": rdir, "deadline_at": deadline_at, "headline_by": headline_by,
               "scale": scale}
        _write_json(os.path.join(d, f"attempt{k}.json"), att)
        t_att = _now()
        child[0] = _spawn(script, att["argv"], _worker_env(att, rdir, 0))
        reason = None
        while True:
            rc = child[0].poll()
            if rc is not None:
                reason = None if rc == 0 else f"rank 0 worker exited with status {rc}"
                break
            res = _read_json(os.path.join(rdir, "result.json"))
            have = res is not None and res.get("value") is not None
            now = _now()
            if now > deadline_at:
                reason = "deadline reached"
                break
            if not have and now > headline_by:
                reason = f"no headline by the attempt's deadline ({headline_by - t_att:.0f} s)"
                break
            bad = [r for r in range(1, world)
                   if (_read_json(os.path.join(d, f"exit{k}_rank{r}.json")) or {}).get("rc")
                   not in (None, 0)]
            if bad and not have:
                # give rank 0's worker a moment to report the failure itself
                try:
                    child[0].wait(timeout=10)
                except subprocess.TimeoutExpired:
                    pass
                reason = f"rank {bad[0]} worker exited with an error"
                break
            time.sleep(poll_s)
        res = _read_json(os.path.join(rdir, "result.json"))
        phases = read_phases(rdir, world)
        rec = dict(rung["label"], attempt=k, seconds=round(_now() - t_att, 1))
        if res is not None and res.get("value") is not None:
            rec["outcome"] = "ok" if res.get("complete") else "ok (extras cut short)"
            if not res.get("complete"):
                res.setdefault("errors", []).append(
                    {"phase": res.get("phase_at_publish"), "error": reason or "worker ended",
                     "stalled_ranks": stalled_ranks(phases)})
            final = res
            code = 4 if (res.get("check") or {}).get("ok") is False else 0
            _kill(child[0])
            attempts.append(rec)
            break
        # no headline: abort this rung on every rank, then fall back
        _write_json(os.path.join(d, f"abort{k}.json"), {"k": k, "nonce": nonce})
        _kill(child[0])
        st = stalled_ranks(phases)
        rec.update(outcome="failed", phase=phases.get(st[0], {}).get("phase") if st else None,
                   stalled_ranks=st, error=(res or {}).get("error") or reason,
                   phases={r: p.get("phase") for r, p in phases.items()})
        attempts.append(rec)
        t_wait = _now() + 20
        while _now() < t_wait and not all(
                os.path.exists(os.path.join(d, f"reaped{k}_rank{r}.json"))
                for r in range(1, world)):
            time.sleep(poll_s)
    if final is None:
        last = attempts[-1] if attempts else {}
        final = dict(base_line, value=None,
                     error=f"no attempt measured the headline: {last.get('error')}",
                     stalled_ranks=last.get("stalled_ranks"), phases=last.get("phases"))
    final.pop("complete", None)
    final.pop("phase_at_publish", None)
    final["attempts"] = attempts
    if len(attempts) > 1 and final.get("value") is not None:
        final["fallback"] = True
    final["supervisor_s"] = round(_now() - t_start, 1)
    print(json.dumps(final), flush=True)
    _write_json(os.path.join(d, "end.json"), {"nonce": nonce, "code": code})
    return code


def _follow(script, rank, world, deadline_s, d, t_start, child, poll_s):
    k, limit = 0, t_start + deadline_s + 60
    fresh = t_start - 120  # files older than this launcher are stale

    def current(name):
        p = os.path.join(d, name)
        try:
            if os.path.getmtime(p) < fresh:
                return None
        except OSError:
            return None
        return _read_json(p)

    nonce = None
    while _now() < limit:
        att = current(f"attempt{k}.json")
        end = current("end.json")
        if end is not None and (nonce is None or end.get("nonce") == nonce):
            return 0
        if att is None:
            time.sleep(poll_s)
            continue
        nonce = att["nonce"]
        child[0] = _spawn(script, att["argv"], _worker_env(att, att["dir"], rank))
        reported = False
        while _now() < limit:
            rc = child[0].poll()
            if rc is not None and not reported:
                _write_json(os.path.join(d, f"exit{k}_rank{rank}.json"), {"rc": rc})
                reported = True
            ab = current(f"abort{k}.json")
            end = current("end.json")
            if (ab is not None and ab.get("nonce") == nonce) or (
                    end is not None and end.get("nonce") == nonce):
                _kill(child[0])
                _write_json(os.path.join(d, f"reaped{k}_rank{rank}.json"), {})
                if end is not None and end.get("nonce") == nonce:
                    return 0
                break
            time.sleep(poll_s)
        k += 1
    _kill(child[0])
    return 3


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
