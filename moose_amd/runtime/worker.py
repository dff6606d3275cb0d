"""Worker process: one identity of a multi-party session (the ``comet`` analogue,
reference ``moose/src/bin/comet/comet.rs:12-83``).

One-shot mode (used by :class:`DistributedMooseRuntime`)::

    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p \\
        python -m moose_amd.runtime.worker --job DIR

reads ``DIR/computation.msgpack`` + ``DIR/job.msgpack``, joins the process group, runs
its party with :func:`moose_amd.runtime.distributed.run_spmd` and writes
``DIR/result_<rank>.msgpack``.  Serve mode (``--serve``) keeps the process group up and
executes sessions posted to the choreography store (see
:mod:`moose_amd.runtime.choreography`).
"""
from __future__ import annotations

import argparse
import os
import sys
import traceback

import numpy as np


def _init_group(backend: str):
    import torch.distributed as dist

    if not dist.is_initialized():
        from datetime import timedelta

        # per-session deadline: a party that never receives (dead peer, dropped message)
        # fails after MOOSEX_SESSION_TIMEOUT seconds instead of hanging
        timeout = timedelta(seconds=float(os.environ.get("MOOSEX_SESSION_TIMEOUT", "1800")))
        dist.init_process_group(backend=backend, timeout=timeout)
    return dist.get_rank(), dist.get_world_size()


def run_job(job: str) -> int:
    import torch
    import torch.distributed as dist

    from moose_amd.ir.computation import Computation
    from moose_amd.runtime.distributed import party_device
    from moose_amd.runtime.distributed import run_spmd
    from moose_amd.utils import valuecodec

    with open(os.path.join(job, "job.msgpack"), "rb") as f:
        spec = valuecodec.loads(f.read())
    with open(os.path.join(job, "computation.msgpack"), "rb") as f:
        comp = Computation.from_msgpack(f.read())
    backend = spec["backend"]
    rank, world = _init_group(backend)
    identities = spec["identities"]
    replicas = int(spec.get("replicas", 1))
    n = len(identities)
    if world != n * replicas:
        raise RuntimeError(f"world size {world} != {n} identities x {replicas} replicas")
    device = party_device(backend, int(os.environ.get("LOCAL_RANK", rank)))
    if device.type == "cuda":
        torch.cuda.set_device(device)
    replica, party = divmod(rank, n)
    ident = identities[party]
    storage = {ident: dict(spec["storage"].get(ident, {}))}
    arguments = dict(spec["arguments"])
    group = owner_groups = None
    if replicas > 1:
        from moose_amd.parallel import replicas as REP

        replica_groups, owner_groups = REP.make_groups(n, replicas)
        group = replica_groups[replica]
        arguments.update(spec["replica_arguments"][replica])
    outs, stats, elapsed = run_spmd(comp, arguments, identities, rank=party,
                                    device=device, seed=spec["seed"],
                                    fixedpoint_ring=spec["fixedpoint_ring"], storage=storage,
                                    group=group, rank_offset=replica * n)
    if replicas > 1:
        comm_dev = device if backend == "nccl" else torch.device("cpu")
        outs = REP.gather_outputs(outs, owner_groups[party], replicas, comm_dev)
        if replica > 0:
            outs = {}
    res = {
        "outputs": {k: np.asarray(v) if not isinstance(v, (str, bytes)) else v
                    for k, v in outs.items()},
        "elapsed_us": elapsed,
        "storage": {k: v for k, v in storage.get(ident, {}).items()
                    if isinstance(v, (np.ndarray, str))},
        "stats": {"rounds": stats.rounds, "reshare_bytes": stats.round_bytes},
    }
    tmp = os.path.join(job, f"result_{rank}.msgpack.tmp")
    with open(tmp, "wb") as f:
        f.write(valuecodec.dumps(res))
    os.replace(tmp, os.path.join(job, f"result_{rank}.msgpack"))
    dist.barrier()
    dist.destroy_process_group()
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--job", help="one-shot job directory")
    ap.add_argument("--serve", action="store_true", help="serve sessions from the store")
    ap.add_argument("--identity", help="serve mode: this worker's identity")
    ap.add_argument("--backend", default=None, help="serve mode: nccl | gloo")
    args = ap.parse_args(argv)
    try:
        if args.job:
            return run_job(args.job)
        if args.serve:
            from moose_amd.runtime.choreography import serve

            return serve(args.identity, args.backend)
        ap.error("one of --job / --serve is required")
    except Exception:
        traceback.print_exc()
        sys.stdout.flush()
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
