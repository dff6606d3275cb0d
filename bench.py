#!/usr/bin/env python
"""Headline benchmark: replicated fixed-point matrix product throughput.

Metric (BASELINE.json): "replicated fixed(14,23) matmul elems/sec" -- one step is the
reference's dot benchmark (``benchmarks/pymoose/dot_product.py``) at the BASELINE config
3 size: x (alice) and y (bob) are cast to fixed(14,23), secret-shared onto a 3-party
replicated placement, multiplied (RSS dot = int8-MFMA limb GEMM + zero share + reshare),
truncated (TruncPr) and revealed to carole, who decodes to float64.  As in pymoose every
fixed dtype runs over Z_2^128 (``--ring 64`` selects the Z_2^64 path).  Value = output
elements per second over the whole job (all GPUs).

Layout: one stacked 3-party session per GPU (all three parties' local work is one
batched kernel per step on that MI355X); N GPUs run N data-parallel session replicas
(weak scaling) and all-gather their revealed outputs over RCCL at the end of each step.
Inputs are synthetic (uniform [-4, 4)), resident on the device; compilation (tracing and
conversion) happens once before the timed region, like the reference's client-side
compile.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

REFERENCE_ELEMS_PER_SEC = 1.0e6 / 5.910  # benchmarks/README.md:21, 1000x1000 Fixed128


def build_computation(ring):
    import moose_amd as pm
    from moose_amd.compiler.from_edsl import convert

    alice = pm.host_placement("alice")
    bob = pm.host_placement("bob")
    carole = pm.host_placement("carole")
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(14, 23)

    @pm.computation
    def dot_product(
        x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64)),
        y: pm.Argument(placement=bob, vtype=pm.TensorType(pm.float64)),
    ):
        with alice:
            xf = pm.cast(x, dtype=fx)
        with bob:
            yf = pm.cast(y, dtype=fx)
        with rep:
            z = pm.dot(xf, yf)
        with carole:
            out = pm.cast(z, dtype=pm.float64)
        return out

    return convert(pm.trace(dot_product), fixedpoint_ring=ring)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--ring", type=int, default=128, choices=[64, 128])
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--layout", default="stacked", choices=["stacked", "spmd"],
                    help="stacked: 3 parties per GPU, N data-parallel sessions (default, "
                         "highest throughput); spmd: each party on its own GPU, N/3 sessions, "
                         "every reshare an RCCL send/recv")
    ap.add_argument("--check", action="store_true", help="verify against float64 numpy")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")
    if world > 1:
        backend = "nccl" if device.type == "cuda" else "gloo"
        dist.init_process_group(backend=backend, device_id=device if device.type == "cuda" else None)

    from moose_amd.runtime.interpreter import Interpreter
    from moose_amd.runtime.session import StackedSession

    comp = build_computation(args.ring)
    n = args.size
    spmd = args.layout == "spmd"
    if spmd and (world < 3 or world % 3):
        raise SystemExit("--layout spmd needs a multiple of 3 GPUs (one per party)")
    n_sessions = world // 3 if spmd else world
    session = rank // 3 if spmd else rank
    g = torch.Generator(device="cpu").manual_seed(1234 + session)
    x = (torch.rand(n, n, generator=g, dtype=torch.float64) * 8 - 4).to(device)
    y = (torch.rand(n, n, generator=g, dtype=torch.float64) * 8 - 4).to(device)
    gather_bufs, gather_group, pending = None, None, []
    if n_sessions > 1 and not args.no_gather:
        # replicas' revealed outputs concatenated along rows (the layout every backend
        # accepts).  Double-buffered: step k's all-gather runs on the RCCL stream while
        # step k+1 computes; a buffer is reused only after its gather completed.
        gather_bufs = [torch.empty((n_sessions * n, n), dtype=torch.float64, device=device)
                       for _ in range(2)]
        if spmd:  # the output owners (carole = party 2) of every session
            gather_group = dist.new_group([3 * s + 2 for s in range(n_sessions)])
    out_owner = (rank % 3 == 2) if spmd else True

    if spmd:
        from moose_amd.parallel.spmd import SPMDSession
        from moose_amd.parallel.transport import Transport

        roles = {r: 3 * session + i for i, r in enumerate(("alice", "bob", "carole"))}
        transport = Transport(rank, world, device)

        def new_session():
            return SPMDSession(("alice", "bob", "carole")[rank % 3], roles, transport, device)
    else:
        def new_session():
            return StackedSession(device)

    n_steps = [0]

    def step():
        sess = new_session()
        interp = Interpreter(sess, {}, fixedpoint_ring=args.ring)
        outs = interp.run(comp, {"x": x, "y": y})
        z = outs["output_0"].v.v if out_owner else None
        if gather_bufs is not None and out_owner:
            if len(pending) == 2:
                pending.pop(0).wait()
            buf = gather_bufs[n_steps[0] % 2]
            pending.append(dist.all_gather_into_tensor(buf, z.contiguous(), group=gather_group,
                                                       async_op=True))
        n_steps[0] += 1
        return z

    def drain():
        while pending:
            pending.pop(0).wait()

    for _ in range(args.warmup):
        step()
    drain()
    if device.type == "cuda":
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        z = step()
    drain()  # every step's gather is complete inside the timed region
    if device.type == "cuda":
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = n_sessions * n * n * args.steps / elapsed

    check = None
    if args.check and out_owner:
        ref = (x.double() @ y.double())
        err = (z - ref).abs().max().item()
        check = {"max_abs_err": err}

    if rank == 0:
        line = {
            "metric": "replicated fixed(14,23) matmul elems/sec",
            "value": value,
            "unit": "output elems/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": value / REFERENCE_ELEMS_PER_SEC,
            "dtype": f"fixed(14,23) over Z_2^{args.ring} (int8-MFMA limb GEMM)",
            "data": "synthetic uniform[-4,4) inputs, device resident",
            "config": {
                "model": f"replicated fixed(14,23) RingDot {n}x{n} (share+dot+trunc_pr+reveal)",
                "global_batch": n_sessions,
                "seq_len": n,
                "parallelism": (f"dp{n_sessions} x 3-party sessions, one party per GPU "
                                "(RCCL reshare)" if spmd else
                                f"dp{world} (one stacked 3-party session per GPU)"),
            },
        }
        if check:
            line["check"] = check
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
