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
* :class:`DistributedMooseRuntime` from a client process: it starts one worker per
  identity on this node (``python -m moose_amd.runtime.worker``) and gathers results.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import tempfile
import time
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
    sess = SPMDSession(identity, role_ranks, tr, device=device, seed=seed)
    interp = Interpreter(sess, store, fixedpoint_ring)
    dist.barrier(group=group)
    t0 = time.perf_counter()
    outs = interp.run(comp, arguments)
    result = {}
    for tag, lv in outs.items():
        if lv.kind == "unit" or not sess.materialized(lv.v):
            continue
        result[tag] = interp.to_numpy(lv)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    elapsed = int((time.perf_counter() - t0) * 1e6)
    return result, sess.stats, elapsed


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
                 replicas: int = 1, shard_args=None, device_map: Optional[List[int]] = None):
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
        for attempt in range(self.retries + 1):
            try:
                return self._launch(comp, dict(arguments or {}))
            except DistributedRuntimeError:
                if attempt == self.retries:
                    raise

    # mirrors pymoose's GrpcMooseRuntime.run_computation -> (outputs, timings)
    def run_computation(self, computation, arguments=None):
        outs = self.evaluate_computation(computation, arguments)
        return outs, dict(self.last_timings or {})

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
        self.storage[identity][key] = np.asarray(value) if not isinstance(value, str) else value


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
