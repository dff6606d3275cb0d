"""Multi-process runtimes: one process per identity, values moved by RCCL (or gloo).

Parity:

* ``GrpcMooseRuntime`` (reference ``pymoose/pymoose/runtime.py:72-139``,
  ``execution/grpc.rs:11-146``): a client launches a computation on a set of workers
  (``comet``) and collects per-role outputs and timings;
* ``AsyncExecutor`` per identity (``execution/asynchronous.rs:557-632``).

MI355X design: each identity is a process bound to its own GPU; all processes of a
session form one ``torch.distributed`` group (backend ``"nccl"`` = RCCL over xGMI, or
``"gloo"`` on CPU) and run the logical computation SPMD-style on a
:class:`~moose_amd.parallel.spmd.SPMDSession` -- protocol steps are fused kernels, every
message is a point-to-point RCCL transfer.  There is no host-op graph to schedule.

Two ways to run:

* :func:`run_spmd` inside an existing process group (e.g. under ``torchrun``);
* :class:`DistributedMooseRuntime` from a client process: it starts one long-running
  worker per identity on this node (``python -m moose_amd.runtime.worker --serve``, the
  ``comet`` analogue) ONCE, then every evaluation is a session posted to their control
  store (:class:`~moose_amd.runtime.choreography.ChoreographyClient`) -- no process start,
  torch import or process-group set-up per evaluation, as the reference's client talks to
  running comet workers (``execution/grpc.rs:46-146``).  ``close()`` shuts them down.
  ``persistent=False`` keeps the one-shot form (fresh workers per evaluation).
"""
from __future__ import annotations

import atexit
import os
import socket
import subprocess
import sys
import tempfile
import time
import uuid
import weakref
from typing import Dict
from typing import List
from typing import Optional

import numpy as np
import torch

from moose_amd import errors
from moose_amd.ir.computation import Computation
from moose_amd.utils import valuecodec


class DistributedRuntimeError(errors.Networking):
    pass


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def party_device(backend: str, local_rank: int) -> torch.device:
    if backend == "nccl":
        return torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
    return torch.device("cpu")


def run_spmd(comp: Computation, arguments: dict, identities: List[str], *, rank: int,
             device=None, seed: Optional[int] = None, fixedpoint_ring: int = 128,
             storage: Optional[dict] = None, group=None, rank_offset: int = 0):
    """Evaluate ``comp`` as party ``identities[rank]`` of an initialised process group.

    ``group``/``rank_offset``: the session runs on a sub-group whose parties are the
    global ranks ``rank_offset + i`` (data-parallel replicas, :mod:`..parallel.replicas`).
    Returns ``(outputs, stats, elapsed_us)`` where ``outputs`` holds the numpy values of
    the outputs this identity owns.
    """
    import torch.distributed as dist

    from moose_amd.parallel.spmd import SPMDSession
    from moose_amd.parallel.transport import Transport
    from moose_amd.runtime.interpreter import Interpreter

    from moose_amd.compiler.passes import is_lowered

    identity = identities[rank]
    role_ranks = {r: rank_offset + i for i, r in enumerate(identities)}
    device = torch.device(device) if device is not None else torch.device("cpu")
    # every worker gets every argument (the client sends them all, as the reference's
    # GrpcMooseRuntime does), so the processes agree on message plans
    tr = Transport(rank_offset + rank, len(identities), device, group=group, plans=True)
    store = storage if storage is not None else {}
    if is_lowered(comp):
        # a compiled host graph: run this identity's operations, Send/Receive over RCCL
        # (the reference's per-identity AsyncExecutor on a lowered computation)
        from moose_amd.runtime.graph_executor import GraphExecutor

        ex = GraphExecutor(device, store, identity=identity, transport=tr, role_ranks=role_ranks)
        dist.barrier(group=group)
        t0 = time.perf_counter()
        raw = ex.run(comp, arguments)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        elapsed = int((time.perf_counter() - t0) * 1e6)
        from moose_amd.utils.telemetry import SessionStats

        return {k: _host_numpy(v) for k, v in raw.items()}, SessionStats(), elapsed
    from moose_amd.parallel import spmd_graphs

    dist.barrier(group=group)
    t0 = time.perf_counter()
    # a program evaluated again with the same argument signature replays its recorded
    # tape (captured kernel segments + prebuilt message rounds, parallel/spmd_graphs.py)
    # a program that Loads: every rank agrees on what the owners' stored values look like
    # (one small collective), so its message plan and tape are keyed on them
    tr.storage_key = (spmd_graphs.storage_key(comp, store, identity, tr, arguments)
                      if getattr(tr, "plans", False) else None)
    taped = spmd_graphs.evaluate(comp, arguments, identity, role_ranks, tr, device, store,
                                 fixedpoint_ring, seed)
    if taped is not None:
        result, stats, _ = taped
    else:
        sess = SPMDSession(identity, role_ranks, tr, device=device, seed=seed)
        interp = Interpreter(sess, store, fixedpoint_ring)
        outs = interp.run(comp, arguments)
        result = {}
        for tag, lv in outs.items():
            if lv.kind == "unit" or not sess.materialized(lv.v):
                continue
            result[tag] = interp.to_numpy(lv)
        stats = sess.stats
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    elapsed = int((time.perf_counter() - t0) * 1e6)
    return result, stats, elapsed


class DistributedMooseRuntime:
    """Client that runs a computation on one worker process per identity.

    ``backend``: ``"nccl"`` (RCCL; one GPU per identity, ``devices`` defaults to
    ``cuda:0..n-1``) or ``"gloo"`` (CPU).  Default: nccl when enough GPUs are visible.
    """

    def __init__(self, identities, backend: Optional[str] = None,
                 storage_mapping: Optional[Dict[str, Dict]] = None, fixedpoint_ring: int = 128,
                 seed: Optional[int] = None, timeout: float = 900.0,
                 master_addr: str = "127.0.0.1", session_timeout: Optional[float] = None,
                 retries: int = 0, worker_env: Optional[Dict[str, str]] = None,
                 replicas: int = 1, shard_args=None, device_map: Optional[List[int]] = None,
                 persistent: bool = True):
        if isinstance(identities, dict):  # GrpcMooseRuntime-style {role: endpoint}
            identities = list(identities.keys())
        self.identities = [getattr(i, "name", i) for i in identities]
        if backend is None:
            n = torch.cuda.device_count() if torch.cuda.is_available() else 0
            backend = "nccl" if n >= len(self.identities) * max(int(replicas), 1) else "gloo"
        self.backend = backend
        self.storage = {i: dict((storage_mapping or {}).get(i, {})) for i in self.identities}
        self.fixedpoint_ring = fixedpoint_ring
        self.seed = seed
        self.timeout = timeout
        self.master_addr = master_addr
        # per-session deadline inside the workers (process-group timeout) and automatic
        # re-launch with a fresh session (new keys, new rendezvous) on failure
        self.session_timeout = session_timeout
        self.retries = retries
        self.worker_env = dict(worker_env or {})
        # data parallelism: `replicas` copies of the session on disjoint GPU groups
        # (global rank = replica * n + party); `shard_args` are split along axis 0 and
        # the outputs concatenated back (parallel/replicas.py).  `device_map[rank]` pins
        # a rank to a GPU index (default: rank).
        self.replicas = int(replicas)
        self.shard_args = list(shard_args or [])
        self.device_map = list(device_map) if device_map is not None else None
        if self.replicas < 1:
            raise ValueError("replicas must be >= 1")
        self.last_timings = None
        self.last_stats = None
        self.last_rounds = None
        # long-running workers (module doc): spawned on first use, reused while their
        # configuration is unchanged, replaced after a failed session
        self.persistent = persistent
        self.worker_spawns = 0
        self._pool = None
        self._sessions = 0
        self._dirty = {i: dict(v) for i, v in self.storage.items() if v}
        _LIVE.add(self)

    def set_default(self):
        from moose_amd.edsl.base import set_current_runtime

        set_current_runtime(self)

    def evaluate_computation(self, computation, arguments=None, compiler_passes=None):
        from moose_amd.runtime.local import to_native

        comp = to_native(computation, self.fixedpoint_ring)
        if compiler_passes:
            from moose_amd.compiler import passes

            from moose_amd.runtime.local import arg_specs_of

            comp = passes.compile(comp, compiler_passes, arg_specs=arg_specs_of(arguments),
                                  fixedpoint_ring=self.fixedpoint_ring)
        launch = self._launch_persistent if self.persistent else self._launch
        for attempt in range(self.retries + 1):
            try:
                return launch(comp, dict(arguments or {}))
            except DistributedRuntimeError:
                if attempt == self.retries:
                    raise

    # mirrors pymoose's GrpcMooseRuntime.run_computation -> (outputs, timings)
    def run_computation(self, computation, arguments=None):
        outs = self.evaluate_computation(computation, arguments)
        return outs, dict(self.last_timings or {})

    # -- persistent workers ---------------------------------------------------------------
    def _pool_key(self):
        return (self.backend, tuple(sorted(self.worker_env.items())), self.session_timeout,
                self.replicas, tuple(self.device_map or ()), self.master_addr)

    def _ensure_pool(self):
        from moose_amd.runtime.choreography import ChoreographyClient

        pool = self._pool
        if pool is not None and pool["key"] == self._pool_key() and all(
                p.poll() is None for p in pool["procs"]):
            return pool
        self.close()
        n = len(self.identities) * self.replicas
        port = free_port()
        env = dict(os.environ)
        for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT", "TORCHELASTIC_USE_AGENT_STORE"):
            env.pop(k, None)
        # MOOSEX_CLIENT_PID: the pool ends with this process even if it never closes it
        env.update(WORLD_SIZE=str(n), MOOSEX_STORE=f"{self.master_addr}:{port}",
                   HSA_ENABLE_IPC_MODE_LEGACY="0", MOOSEX_CLIENT_PID=str(os.getpid()))
        if self.session_timeout is not None:
            env["MOOSEX_SESSION_TIMEOUT"] = str(self.session_timeout)
        env.update(self.worker_env)
        pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = pkg_root + os.pathsep + env.get("PYTHONPATH", "")
        logdir = tempfile.mkdtemp(prefix="moosex_workers_")
        procs, logs = [], []
        for r in range(n):
            dev = self.device_map[r] if self.device_map is not None else r
            log = open(os.path.join(logdir, f"worker{r}.log"), "wb")
            logs.append(log)
            procs.append(subprocess.Popen(
                [sys.executable, "-m", "moose_amd.runtime.worker", "--serve",
                 "--identity", self.identities[r % len(self.identities)],
                 "--backend", self.backend],
                env=dict(env, RANK=str(r), LOCAL_RANK=str(dev)), stdout=log,
                stderr=subprocess.STDOUT))
        self.worker_spawns += 1
        pool = {"key": self._pool_key(), "procs": procs, "logs": logs, "logdir": logdir,
                "client": None}
        self._pool = pool
        deadline = time.time() + min(self.timeout, 600)
        while True:  # rank 0 hosts the store; the client connects once it is up
            if any(p.poll() is not None for p in procs):
                raise DistributedRuntimeError(f"a worker exited during start-up:\n"
                                              f"{self._worker_logs()}")
            try:
                pool["client"] = ChoreographyClient(f"{self.master_addr}:{port}", timeout=30)
                break
            except Exception:  # noqa: BLE001 - not listening yet
                if time.time() > deadline:
                    raise DistributedRuntimeError("workers did not start") from None
                time.sleep(0.2)
        client = pool["client"]
        from moose_amd.runtime.choreography import PREFIX
        from moose_amd.runtime.choreography import _has

        for r in range(n):  # every worker registered: the process group is up
            while not _has(client.store, f"{PREFIX}/worker/{r}"):
                if any(p.poll() is not None for p in procs) or time.time() > deadline:
                    raise DistributedRuntimeError(f"worker {r} did not register:\n"
                                                  f"{self._worker_logs()}")
                time.sleep(0.05)
        # fresh workers hold no storage: everything the client knows goes with the next job
        self._dirty = {i: dict(v) for i, v in self.storage.items() if v}
        return pool

    def _worker_logs(self, tail=3000):
        pool = self._pool
        if pool is None:
            return ""
        out = []
        for r, lg in enumerate(pool["logs"]):
            try:
                lg.flush()
                with open(lg.name, "rb") as f:
                    out.append(f"--- worker {r}\n" + f.read().decode(errors="replace")[-tail:])
            except OSError:
                pass
        return "\n".join(out)

    def _launch_persistent(self, comp: Computation, arguments: dict):
        R = self.replicas
        n = len(self.identities) * R
        replica_args = None
        if R > 1:
            from moose_amd.parallel.replicas import shard_arguments

            shards = shard_arguments(arguments, self.shard_args, R)
            arguments = {k: v for k, v in arguments.items() if k not in self.shard_args}
            replica_args = [{k: v for k, v in sh.items() if k in self.shard_args}
                            for sh in shards]
        pool = self._ensure_pool()
        client = pool["client"]
        self._sessions += 1
        sid = f"{os.getpid()}-{self._sessions}-{uuid.uuid4().hex[:8]}"
        job = {"session_id": sid, "computation": comp.to_msgpack(),
               "arguments": _encodable(arguments), "identities": self.identities,
               "fixedpoint_ring": self.fixedpoint_ring, "seed": self.seed, "replicas": R,
               "replica_arguments": [_encodable(a) for a in replica_args or []],
               "storage_update": {k: _encodable(v) for k, v in self._dirty.items() if v},
               "by_rank": True}
        client.post_job(job)
        self._dirty = {}
        deadline = time.time() + self.timeout
        results, pending = {}, set(range(n))
        try:
            while pending:
                for r in sorted(pending):
                    res = client.result(sid, r, wait_s=0.5)  # blocks on the store
                    if res is None:
                        break
                    results[r] = res
                    pending.discard(r)
                if not pending:
                    break
                dead = [r for r, p in enumerate(pool["procs"]) if p.poll() is not None]
                if dead:
                    raise DistributedRuntimeError(
                        f"worker(s) {dead} exited during session {sid}:\n{self._worker_logs()}")
                if time.time() > deadline:
                    raise DistributedRuntimeError(f"session {sid} timed out after "
                                                  f"{self.timeout:.0f} s (workers {sorted(pending)})")
            failed = {r: res for r, res in results.items() if "error" in res}
            if failed:
                msg = "\n".join(f"--- {self.identities[r % len(self.identities)]} rank {r}: "
                                f"{res['error']}\n{res.get('trace', '')[-2000:]}"
                                for r, res in sorted(failed.items()))
                raise DistributedRuntimeError(f"worker(s) failed:\n{msg}")
        except DistributedRuntimeError:
            self.close()  # a failed session may leave the process group unusable
            raise
        outputs, timings = {}, {}
        for r in range(n):
            ident = self.identities[r % len(self.identities)]
            res = results[r]
            outputs.update(res["outputs"])  # replica 0 holds the gathered outputs
            timings[ident] = max(timings.get(ident, 0), res["elapsed_us"])
            if r < len(self.identities):
                self.storage[ident].update(res.get("storage", {}))
        self.last_timings = timings
        self.last_rounds = max(res.get("rounds", 0) for res in results.values())
        return outputs

    def close(self):
        """Shut the long-running workers down (they finish the session they run)."""
        pool, self._pool = self._pool, None
        if pool is None:
            return
        try:
            if pool["client"] is not None and all(p.poll() is None for p in pool["procs"]):
                pool["client"].shutdown()
        except Exception:  # noqa: BLE001 - the store may be gone with a dead rank 0
            pass
        for p in pool["procs"]:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for lg in pool["logs"]:
            lg.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        # a runtime dropped without close(): its pool must not outlive it (the workers also
        # watch MOOSEX_CLIENT_PID, but only for the client process's exit)
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def _launch(self, comp: Computation, arguments: dict):
        R = self.replicas
        n = len(self.identities) * R
        replica_args = None
        if R > 1:
            from moose_amd.parallel.replicas import shard_arguments

            shards = shard_arguments(arguments, self.shard_args, R)
            arguments = {k: v for k, v in arguments.items() if k not in self.shard_args}
            replica_args = [{k: v for k, v in sh.items() if k in self.shard_args}
                            for sh in shards]
        with tempfile.TemporaryDirectory(prefix="moosex_job_") as job:
            with open(os.path.join(job, "computation.msgpack"), "wb") as f:
                f.write(comp.to_msgpack())
            with open(os.path.join(job, "job.msgpack"), "wb") as f:
                f.write(valuecodec.dumps({
                    "identities": self.identities,
                    "arguments": _encodable(arguments),
                    "storage": {k: _encodable(v) for k, v in self.storage.items()},
                    "fixedpoint_ring": self.fixedpoint_ring,
                    "seed": self.seed,
                    "backend": self.backend,
                    "replicas": R,
                    "replica_arguments": [_encodable(a) for a in replica_args or []],
                }))
            port = free_port()
            env = dict(os.environ)
            env.update(MASTER_ADDR=self.master_addr, MASTER_PORT=str(port),
                       WORLD_SIZE=str(n), HSA_ENABLE_IPC_MODE_LEGACY="0")
            if self.session_timeout is not None:
                env["MOOSEX_SESSION_TIMEOUT"] = str(self.session_timeout)
            env.update(self.worker_env)
            pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            env["PYTHONPATH"] = pkg_root + os.pathsep + env.get("PYTHONPATH", "")
            procs = []
            for r in range(n):
                dev = self.device_map[r] if self.device_map is not None else r
                e = dict(env, RANK=str(r), LOCAL_RANK=str(dev))
                procs.append(subprocess.Popen(
                    [sys.executable, "-m", "moose_amd.runtime.worker", "--job", job],
                    env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
            logs, failed = [], []
            deadline = time.time() + self.timeout
            for r, p in enumerate(procs):
                try:
                    out, _ = p.communicate(timeout=max(1.0, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    for q in procs:
                        q.kill()
                    raise DistributedRuntimeError(
                        f"worker {self.identities[r % len(self.identities)]} timed out")
                logs.append(out.decode(errors="replace"))
                if p.returncode != 0:
                    failed.append(r)
            if failed:
                msg = "\n".join(f"--- {self.identities[r % len(self.identities)]} rank {r} "
                                f"(rc={procs[r].returncode})\n{logs[r][-3000:]}"
                                for r in failed)
                raise DistributedRuntimeError(f"worker(s) failed:\n{msg}")
            outputs, timings = {}, {}
            for r in range(n):
                ident = self.identities[r % len(self.identities)]
                with open(os.path.join(job, f"result_{r}.msgpack"), "rb") as f:
                    res = valuecodec.loads(f.read())
                outputs.update(res["outputs"])  # replica 0 holds the gathered outputs
                timings[ident] = max(timings.get(ident, 0), res["elapsed_us"])
                if r < len(self.identities):
                    self.storage[ident].update(res.get("storage", {}))
            self.last_timings = timings
            return outputs

    def read_value_from_storage(self, identity, key):
        return self.storage[identity][key]

    def write_value_to_storage(self, identity, key, value):
        v = np.asarray(value) if not isinstance(value, str) else value
        self.storage[identity][key] = v
        self._dirty.setdefault(identity, {})[key] = v  # reaches the worker with the next job


_LIVE: "weakref.WeakSet" = weakref.WeakSet()


@atexit.register
def _close_all():
    for rt in list(_LIVE):
        try:
            rt.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def _host_numpy(v):
    """Output value of a lowered graph -> numpy (ring tensors as integers)."""
    from moose_amd.ops import ring as R

    if isinstance(v, R.RT):
        return np.asarray(R.to_ints(v))
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().numpy()
    return v


def _encodable(d: dict) -> dict:
    out = {}
    for k, v in d.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        elif isinstance(v, (list, float, int)) and not isinstance(v, bool):
            v = np.asarray(v) if isinstance(v, list) else v
        out[k] = v
    return out


# the reference's client runtime name; the control plane here is a local process launcher
GrpcMooseRuntime = DistributedMooseRuntime
