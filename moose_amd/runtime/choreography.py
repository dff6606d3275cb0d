"""Choreography: long-running party workers that execute sessions on request.

Parity:

* gRPC choreography + ``comet`` worker (``choreography/grpc.rs:34-233``,
  ``bin/comet/comet.rs``): ``launch_computation`` (duplicate session ids rejected),
  ``retrieve_results`` (blocks until done, returns outputs + elapsed time),
  ``abort_computation``;
* ``cometctl`` client (``bin/comet/cometctl.rs``) and ``GrpcMooseRuntime``;
* filesystem choreography (``choreography/filesystem.rs:28-259``, ``rudolph``): a
  directory of ``<session-id>.session`` TOML files (``[computation] path, format`` and
  ``[[roles]] name, endpoint``) is watched and every new file is launched.

MI355X design: the control plane is a ``torch.distributed.TCPStore`` (native C++
key-value server hosted by worker rank 0); the data plane is the workers' process
group (RCCL between GPUs, gloo on CPU) -- the same one the SPMD session uses, so a
session costs no connection setup.  Keys::

    moosex/worker/<rank>            -> identity of that worker
    moosex/launch_count             -> number of launched sessions (atomic add)
    moosex/session/<n>              -> n-th job (valuecodec: sid, computation, args, ...)
    moosex/result/<sid>/<identity>  -> that identity's outputs / error / elapsed_us
    moosex/abort/<sid>              -> abort request
"""
from __future__ import annotations

import glob
import os
import threading
import time
import traceback
from datetime import timedelta
from typing import Dict
from typing import List
from typing import Optional

import numpy as np

from moose_amd import errors
from moose_amd.utils import valuecodec

PREFIX = "moosex"


def _store(addr: str, is_master: bool, world: Optional[int] = None, timeout=3600):
    import torch.distributed as dist

    host, _, port = addr.rpartition(":")
    return dist.TCPStore(host or "127.0.0.1", int(port), world_size=world, is_master=is_master,
                         timeout=timedelta(seconds=timeout), wait_for_workers=False)


def _get(store, key: str) -> bytes:
    return bytes(store.get(key))


def _has(store, key: str) -> bool:
    return store.check([key])


# ---------------------------------------------------------------------------
# worker
# ---------------------------------------------------------------------------
class Worker:
    """One identity of a group of choreographed workers (rank 0 hosts the store)."""

    def __init__(self, identity: str, rank: int, world: int, store_addr: str,
                 backend: str = "gloo", storage_dir: Optional[str] = None):
        import torch
        import torch.distributed as dist

        from moose_amd.runtime.distributed import party_device

        self.identity = identity
        self.rank = rank
        self.world = world
        self.store = _store(store_addr, rank == 0, world)
        self.store.set(f"{PREFIX}/worker/{rank}", identity)
        self.backend = backend
        self.device = party_device(backend, int(os.environ.get("LOCAL_RANK", rank)))
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        if not dist.is_initialized():
            # per-session deadline: a party that never receives (dead peer, dropped
            # message) fails after MOOSEX_SESSION_TIMEOUT seconds instead of hanging
            tmo = timedelta(seconds=float(os.environ.get("MOOSEX_SESSION_TIMEOUT", "1800")))
            dist.init_process_group(backend, store=dist.PrefixStore("pg", self.store),
                                    rank=rank, world_size=world, timeout=tmo)
        self.identities = [_get(self.store, f"{PREFIX}/worker/{r}").decode() for r in range(world)]
        self.storage_dir = storage_dir
        self.storage: Dict[str, object] = {}
        self.seen = set()
        self._groups = {}  # (parties, replicas) -> replica / owner process groups

    def serve(self, max_sessions: Optional[int] = None, poll_s: float = 0.05) -> int:
        """Run jobs until a shutdown job.  A pool started for one client
        (``MOOSEX_CLIENT_PID``, DistributedMooseRuntime) also ends when that client is gone
        -- it may exit without closing the pool -- and any worker ends when the store it
        waits on is unreachable (rank 0, which hosts it, died)."""
        client = int(os.environ.get("MOOSEX_CLIENT_PID", "0") or 0)
        if client:
            _die_with(client)
        n = 0
        while max_sessions is None or n < max_sessions:
            key = f"{PREFIX}/session/{n}"
            while True:  # block on the store (no polling latency per session)
                t0 = time.monotonic()
                try:
                    self.store.wait([key], timedelta(seconds=5.0 if client else 30.0))
                    break
                except Exception:  # noqa: BLE001 - a timeout, or a dead store
                    if client and not _alive(client):
                        return 0
                    if time.monotonic() - t0 < 1.0:  # failed at once: the store is gone
                        if not _store_alive(self.store):
                            return 0
                        time.sleep(0.5)
                    continue
            job = valuecodec.loads(_get(self.store, key))
            n += 1
            if job.get("shutdown"):
                break
            self._run(job)
        return 0

    def _run(self, job):
        """One session.  Besides the reference's launch fields a job may carry (the
        :class:`~moose_amd.runtime.distributed.DistributedMooseRuntime` client):
        ``identities`` (party order), ``replicas`` + ``replica_arguments`` (data-parallel
        copies of the session, global rank = replica * parties + party), ``seed``,
        ``storage_update`` (values the client wrote to this identity's storage) and
        ``by_rank`` (results keyed by rank: replicas share identities)."""
        import torch
        import torch.distributed as dist

        from moose_amd.ir.computation import Computation
        from moose_amd.runtime.distributed import run_spmd

        sid = job["session_id"]
        rkey = f"{PREFIX}/result/{sid}/{self.rank if job.get('by_rank') else self.identity}"
        if sid in self.seen:  # choreography/grpc.rs:114-118
            self.store.set(rkey, valuecodec.dumps({"error": f"session {sid} already exists"}))
            return
        self.seen.add(sid)
        # rank 0 decides whether an abort request arrived before the start, so every
        # worker takes the same branch
        flag = torch.tensor([1 if (self.rank == 0 and _has(self.store, f"{PREFIX}/abort/{sid}"))
                             else 0], device=self.device)
        dist.broadcast(flag, 0)
        if int(flag.item()):
            self.store.set(rkey, valuecodec.dumps({"error": "aborted"}))
            return
        try:
            comp = Computation.from_msgpack(job["computation"])
            replicas = int(job.get("replicas", 1))
            if job.get("identities"):
                idents = list(job["identities"])
            else:
                roles = job.get("role_assignment") or {}
                # identities in rank order, renamed to the computation's roles
                inv = {ident: role for role, ident in roles.items()}
                idents = [inv.get(i, i) for i in self.identities]
            n = len(idents)
            if n * replicas != self.world:
                raise RuntimeError(f"{n} identities x {replicas} replicas != {self.world} workers")
            replica, party = divmod(self.rank, n)
            me = idents[party]
            upd = (job.get("storage_update") or {}).get(me)
            if upd:
                self._save_storage(upd)
            mine = self._load_storage()
            before = dict(mine)
            storage = {me: mine}
            arguments = dict(job.get("arguments", {}))
            group = owner_groups = None
            if replicas > 1:
                from moose_amd.parallel import replicas as REP

                if (n, replicas) not in self._groups:  # every worker, same order
                    self._groups[(n, replicas)] = REP.make_groups(n, replicas)
                replica_groups, owner_groups = self._groups[(n, replicas)]
                group = replica_groups[replica]
                arguments.update((job.get("replica_arguments") or [{}] * replicas)[replica])
            outs, stats, elapsed = run_spmd(comp, arguments, idents, rank=party,
                                            device=self.device, seed=job.get("seed"),
                                            fixedpoint_ring=job.get("fixedpoint_ring", 128),
                                            storage=storage, group=group,
                                            rank_offset=replica * n)
            if replicas > 1:
                comm_dev = self.device if self.backend == "nccl" else torch.device("cpu")
                outs = REP.gather_outputs(outs, owner_groups[party], replicas, comm_dev)
                if replica > 0:
                    outs = {}
            saved = {k: v for k, v in storage.get(me, {}).items()
                     if before.get(k) is not v and isinstance(v, (np.ndarray, str))}
            self._save_storage(saved)
            res = {"outputs": {k: np.asarray(v) if not isinstance(v, (str, bytes)) else v
                               for k, v in outs.items()},
                   "elapsed_us": elapsed, "rounds": stats.rounds, "storage": saved}
        except Exception as e:  # report, keep serving
            res = {"error": f"{type(e).__name__}: {e}", "trace": traceback.format_exc()[-4000:]}
        self.store.set(rkey, valuecodec.dumps(res))

    def _load_storage(self):
        if self.storage_dir is None:
            return dict(self.storage)
        from moose_amd.utils.storage import load_from_path

        out = {}
        for p in glob.glob(os.path.join(self.storage_dir, "*.npy")):
            out[os.path.basename(p)[:-4]] = load_from_path(p)
        return out

    def _save_storage(self, store):
        for k, v in store.items():
            if self.storage_dir is None:
                self.storage[k] = v
            elif isinstance(v, np.ndarray):
                np.save(os.path.join(self.storage_dir, f"{k}.npy"), v, allow_pickle=False)


# ---------------------------------------------------------------------------
# client
# ---------------------------------------------------------------------------
class ChoreographyClient:
    """``cometctl`` / ``GrpcMooseRuntime`` analogue talking to the workers' store."""

    def __init__(self, store_addr: str, timeout: float = 3600):
        self.store = _store(store_addr, False, None, timeout)
        self.timeout = timeout

    def worker_identities(self, world: int) -> List[str]:
        return [_get(self.store, f"{PREFIX}/worker/{r}").decode() for r in range(world)]

    def post_job(self, job: dict) -> int:
        """Queue a prepared job (``Worker._run`` fields) for every worker; returns its
        index.  Duplicate session ids are rejected (choreography/grpc.rs:114-118)."""
        if self.store.add(f"{PREFIX}/sid/{job['session_id']}", 1) > 1:
            raise errors.SessionAlreadyExists(f"session {job['session_id']} already exists")
        n = self.store.add(f"{PREFIX}/launch_count", 1) - 1
        self.store.set(f"{PREFIX}/session/{n}", valuecodec.dumps(job))
        return n

    def result(self, session_id: str, who, wait_s: float = 0.0) -> Optional[dict]:
        """One worker's result record (keyed by identity, or by rank for ``by_rank``
        jobs), or None if it is not there within ``wait_s`` seconds."""
        key = f"{PREFIX}/result/{session_id}/{who}"
        if not _has(self.store, key):
            if wait_s <= 0:
                return None
            try:
                self.store.wait([key], timedelta(seconds=wait_s))
            except Exception:  # noqa: BLE001 - not yet
                return None
        return valuecodec.loads(_get(self.store, key))

    def launch_computation(self, session_id: str, computation, arguments=None,
                           role_assignment=None, fixedpoint_ring: int = 128):
        from moose_amd.runtime.local import to_native

        if self.store.add(f"{PREFIX}/sid/{session_id}", 1) > 1:  # choreography/grpc.rs:114
            raise errors.SessionAlreadyExists(f"session {session_id} already exists")
        comp = to_native(computation, fixedpoint_ring)
        job = {"session_id": str(session_id), "computation": comp.to_msgpack(),
               "arguments": _plain_args(arguments or {}),
               "role_assignment": dict(role_assignment or {}),
               "fixedpoint_ring": fixedpoint_ring}
        n = self.store.add(f"{PREFIX}/launch_count", 1) - 1
        self.store.set(f"{PREFIX}/session/{n}", valuecodec.dumps(job))
        return n

    def retrieve_results(self, session_id: str, identities: List[str], timeout=None):
        deadline = time.time() + (timeout or self.timeout)
        outputs, timings = {}, {}
        for ident in identities:
            key = f"{PREFIX}/result/{session_id}/{ident}"
            while not _has(self.store, key):
                if time.time() > deadline:
                    raise TimeoutError(f"no result from {ident} for session {session_id}")
                time.sleep(0.05)
            res = valuecodec.loads(_get(self.store, key))
            if "error" in res:
                raise RuntimeError(f"{ident}: {res['error']}\n{res.get('trace', '')}")
            outputs.update(res["outputs"])
            timings[ident] = res["elapsed_us"]
        return outputs, timings

    def abort_computation(self, session_id: str):
        self.store.set(f"{PREFIX}/abort/{session_id}", b"1")

    def run_computation(self, session_id, computation, arguments, identities, role_assignment=None):
        self.launch_computation(session_id, computation, arguments, role_assignment)
        return self.retrieve_results(session_id, identities)

    def shutdown(self):
        n = self.store.add(f"{PREFIX}/launch_count", 1) - 1
        self.store.set(f"{PREFIX}/session/{n}", valuecodec.dumps({"shutdown": True}))


def _die_with(pid: int):
    """Exit at once if the client ``pid`` (this process's parent) is already gone; the serve
    loop checks again at every 5 s wait.  (No PR_SET_PDEATHSIG: it fires when the parent
    THREAD that spawned the pool exits, which may be long before the client does.)"""
    if not _alive(pid):
        os._exit(0)


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return os.getppid() == pid


def _store_alive(store) -> bool:
    try:
        store.check([f"{PREFIX}/alive"])
        return True
    except Exception:  # noqa: BLE001
        return False


def _plain_args(d):
    import torch

    out = {}
    for k, v in d.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        elif isinstance(v, list):
            v = np.asarray(v)
        out[k] = v
    return out


# ---------------------------------------------------------------------------
# filesystem choreography
# ---------------------------------------------------------------------------
def parse_session_file(path: str) -> dict:
    """``[computation] path = ..., format = "textual"|"msgpack"`` and
    ``[[roles]] name = ..., endpoint = ...`` (reference examples/test.session), plus the
    GPU topology of this engine (optional):

    * ``[[roles]] gpu = g`` -- the device ordinal (on its endpoint's node) that runs the
      role in replica 0; ``gpus = [g0, g1, ...]`` -- one per replica;
    * ``[session] replicas = R`` -- data-parallel copies of the 3-party session on
      disjoint GPU groups; ``shard_args = ["x", ...]`` -- arguments split along axis 0
      across the replicas (outputs concatenated back, parallel/replicas.py);
      ``fixedpoint_ring = 64|128``; ``[arguments] name = "file.npy"``.
    """
    import tomli

    with open(path, "rb") as f:
        d = tomli.load(f)
    base = os.path.dirname(os.path.abspath(path))
    comp = d.get("computation", {})
    cpath = comp["path"]
    if not os.path.isabs(cpath):
        cpath = os.path.join(base, cpath)
    role_list = d.get("roles", [])
    roles = {r["name"]: r.get("endpoint", r["name"]) for r in role_list}
    sess = d.get("session", {})
    replicas = int(sess.get("replicas", 1))
    if replicas < 1:
        raise ValueError(f"{path}: replicas must be >= 1")
    gpus = {}
    for i, r in enumerate(role_list):
        if "gpus" in r:
            g = [int(v) for v in r["gpus"]]
            if len(g) != replicas:
                raise ValueError(f"{path}: role {r['name']} lists {len(g)} gpus for "
                                 f"{replicas} replicas")
            gpus[r["name"]] = g
        elif "gpu" in r:
            gpus[r["name"]] = [int(r["gpu"]) + k * len(role_list) for k in range(replicas)]
    args = {k: (v if os.path.isabs(v) else os.path.join(base, v))
            for k, v in d.get("arguments", {}).items()}
    return {"session_id": os.path.splitext(os.path.basename(path))[0],
            "computation_path": cpath, "format": comp.get("format", "textual"), "roles": roles,
            "replicas": replicas, "shard_args": list(sess.get("shard_args", [])),
            "fixedpoint_ring": int(sess.get("fixedpoint_ring", 128)), "gpus": gpus,
            "arguments": args}


def session_device_map(s: dict) -> Optional[List[int]]:
    """Global rank -> device ordinal for a parsed session (rank = replica * n + role
    index, roles in file order), or None when the file pins no GPU."""
    if not s["gpus"]:
        return None
    names = list(s["roles"])
    n = len(names)
    dm = []
    for k in range(s["replicas"]):
        for i, name in enumerate(names):
            g = s["gpus"].get(name)
            dm.append(g[k] if g is not None else k * n + i)
    if len(set(dm)) != len(dm):
        raise ValueError(f"session {s['session_id']}: two ranks pinned to one GPU: {dm}")
    return dm


def run_session_file(path: str, arguments: Optional[dict] = None, backend=None, **kw):
    """Run a ``.session`` file on one node as one worker process per (replica, role),
    honouring its GPU pinning and replicas (DistributedMooseRuntime); returns
    (outputs, timings)."""
    from moose_amd.cli.common import read_computation
    from moose_amd.runtime.distributed import DistributedMooseRuntime
    from moose_amd.utils.storage import load_from_path

    s = parse_session_file(path)
    comp = read_computation(s["computation_path"], s["format"])
    args = {k: load_from_path(v, None) for k, v in s["arguments"].items()}
    args.update(arguments or {})
    rt = DistributedMooseRuntime(list(s["roles"]), backend=backend,
                                 fixedpoint_ring=s["fixedpoint_ring"], replicas=s["replicas"],
                                 shard_args=s["shard_args"] or None,
                                 device_map=session_device_map(s), **kw)
    return rt.run_computation(comp, args)


def watch_sessions(sessions_dir: str, client: ChoreographyClient, world: int,
                   stop: threading.Event, poll_s: float = 0.2, log=print,
                   ignore_existing: bool = False, no_listen: bool = False):
    """Launch every new ``*.session`` file in ``sessions_dir`` (session id = stem) and log
    its outputs when done (choreography/filesystem.rs).  ``ignore_existing``: only files
    that appear after start-up; ``no_listen``: process the existing files once, then shut
    the workers down (rudolph ``--ignore-existing`` / ``--no-listen``, main.rs:29-37)."""
    from moose_amd.cli.common import read_computation

    pattern = os.path.join(sessions_dir, "*.session")
    launched = set(glob.glob(pattern)) if ignore_existing else set()
    idents = client.worker_identities(world)
    while not stop.is_set():
        for p in sorted(glob.glob(pattern)):
            if p in launched:
                continue
            launched.add(p)
            try:
                s = parse_session_file(p)
                comp = read_computation(s["computation_path"], s["format"])
                # roles are mapped to the workers whose identity is the role's endpoint name
                ra = {role: ep.split(":")[0] if ep not in idents else ep
                      for role, ep in s["roles"].items()}
                ra = {role: (ident if ident in idents else role) for role, ident in ra.items()}
                client.launch_computation(s["session_id"], comp, {}, ra)
                outs, timings = client.retrieve_results(s["session_id"], idents)
                log(f"session {s['session_id']}: outputs {sorted(outs)} timings {timings}")
                for k, v in outs.items():
                    np.save(os.path.join(sessions_dir, f"{s['session_id']}.{k}.npy"),
                            np.asarray(v), allow_pickle=False)
            except Exception as e:
                log(f"session {os.path.basename(p)} failed: {e}")
        if no_listen:
            client.shutdown()
            return
        stop.wait(poll_s)


def serve(identity: Optional[str], backend: Optional[str]) -> int:
    """Entry used by ``python -m moose_amd.runtime.worker --serve`` (env: RANK,
    WORLD_SIZE, MOOSEX_STORE=host:port)."""
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    addr = os.environ.get("MOOSEX_STORE", "127.0.0.1:29600")
    w = Worker(identity or f"worker{rank}", rank, world, addr, backend or "gloo")
    return w.serve()
