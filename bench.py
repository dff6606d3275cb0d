#!/usr/bin/env python
"""Headline benchmark: replicated fixed-point matrix product throughput.

Metric (BASELINE.json): "replicated fixed(14,23) matmul elems/sec" -- one step is the
reference's dot benchmark (``benchmarks/pymoose/dot_product.py``) at the BASELINE config
3 size: x (alice) and y (bob) are cast to fixed(14,23), secret-shared onto a 3-party
replicated placement, multiplied (RSS dot = exact multi-modular int8-MFMA GEMM + zero share
+ reshare),
truncated (TruncPr) and revealed to carole, who decodes to float64.  As in pymoose every
fixed dtype runs over Z_2^128 (``--ring 64`` selects the Z_2^64 path).  Value = output
elements per second over the whole job (all GPUs).

Layouts (``--layout``; default ``auto`` = stacked on 1 GPU, cyclic on N > 1):

* ``stacked`` -- one 3-party session per GPU, all three parties' local work batched into
  one kernel per protocol step; N GPUs = N data-parallel session replicas.
* ``cyclic`` -- N sessions on N GPUs, every party of a session on a DIFFERENT GPU (role r
  of session s on GPU (s + r) mod N, ``moose_amd/parallel/cyclic.py``): each GPU does one
  session's worth of work and every reshare / dealer message / reveal is an RCCL
  send/recv over xGMI.  Weak scaling with the same per-GPU work as the 1-GPU stacked run.
* ``spmd`` -- one party per GPU, N/3 sessions (latency layout).

With several sessions, the revealed outputs of every session are collected on rank 0 (the
client, as the reference's benchmark collects them) over RCCL inside the timed region,
overlapped with the next step (``--gather all`` all-gathers them to every rank instead).  Inputs are synthetic (uniform [-4, 4)),
device-resident; tracing/conversion happens once before the timed region (the
reference's client-side compile).  Every step creates a fresh session (fresh PRF keys).

Launch: ``python bench.py --gpus N`` spawns N ranks itself (torch.distributed.run on
127.0.0.1, before anything touches the GPU); under an external launcher (WORLD_SIZE set)
it runs as one rank.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

REFERENCE_ELEMS_PER_SEC = 1.0e6 / 5.910  # benchmarks/README.md:21, 1000x1000 Fixed128
ROLES = ("alice", "bob", "carole")


def build_computation(ring):
    import moose_amd as pm
    from moose_amd.compiler.from_edsl import convert

    alice, bob, carole = (pm.host_placement(r) for r in ROLES)
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


def _parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--ring", type=int, default=128, choices=[64, 128])
    ap.add_argument("--gather", default="root", choices=["root", "all", "none"],
                    help="revealed outputs of every session: to rank 0 (the client; "
                         "default), all-gathered to every rank, or left on their owners")
    ap.add_argument("--no-gather", action="store_true", help="= --gather none")
    ap.add_argument("--layout", default="auto", choices=["auto", "stacked", "cyclic", "spmd"])
    ap.add_argument("--check", action="store_true", help="verify against float64 torch")
    return ap.parse_args()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(args):
    """N > 1 without a launcher: run N fresh ranks as child processes.  This process has
    not touched the GPU (only argparse ran), and exits with the launcher's status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _device_info(device):
    """Identity of the GPU the numbers were taken on (and the torch/HIP/RCCL versions)."""
    import torch

    info = {"torch": torch.__version__, "hip": torch.version.hip}
    if device.type != "cuda":
        return dict(info, name="cpu")
    p = torch.cuda.get_device_properties(device)
    info.update(name=p.name, arch=getattr(p, "gcnArchName", ""),
                cus=p.multi_processor_count, mem_gib=round(p.total_memory / 2**30, 1),
                clock_mhz=getattr(p, "clock_rate", 0) // 1000 or None)
    try:
        v = torch.cuda.nccl.version()
        info["rccl"] = ".".join(map(str, v)) if isinstance(v, tuple) else v
    except Exception:  # noqa: BLE001 - informational only
        pass
    return info


def _revision():
    """git head of the tree (the GPU box gets a snapshot without .git: fall back to the
    REVISION file written by __graft_entry__.build())."""
    here = os.path.dirname(os.path.abspath(__file__))
    try:
        return subprocess.run(["git", "-C", here, "rev-parse", "--short=12", "HEAD"],
                              capture_output=True, text=True, timeout=5,
                              check=True).stdout.strip()
    except Exception:  # noqa: BLE001
        try:
            with open(os.path.join(here, "moose_amd", "_native", "REVISION")) as f:
                return f.read().strip()
        except OSError:
            return None


def _inputs(n, session, which, device):
    import torch

    g = torch.Generator(device="cpu").manual_seed(1234 + 2 * session + (which == "y"))
    return (torch.rand(n, n, generator=g, dtype=torch.float64) * 8 - 4).to(device)


def main():
    args = _parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started {world} ranks")
    # MOOSEX_SHARED_GPU=1: every rank on cuda:0 with gloo (rehearsing the multi-GPU
    # layouts on a one-GPU box; RCCL refuses two ranks on one device)
    shared = os.environ.get("MOOSEX_SHARED_GPU") == "1"
    if torch.cuda.is_available():
        idx = 0 if shared else local_rank
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    if world > 1:
        backend = "nccl" if device.type == "cuda" and not shared else "gloo"
        dist.init_process_group(backend=backend,
                                device_id=device if backend == "nccl" else None)
        dist.barrier()

    from moose_amd.runtime.interpreter import Interpreter
    from moose_amd.runtime.session import StackedSession

    layout = args.layout
    if layout == "auto":
        layout = "stacked" if world == 1 else "cyclic"
    if layout == "spmd" and (world < 3 or world % 3):
        raise SystemExit("--layout spmd needs a multiple of 3 GPUs (one per party)")

    comp = build_computation(args.ring)
    n = args.size
    if layout == "spmd":
        n_sessions, out_owner = world // 3, rank % 3 == 2
        xs, ys, out_session = rank // 3, rank // 3, rank // 3
    elif layout == "cyclic":  # rank g hosts alice of session g, bob of g-1, carole of g-2
        n_sessions, out_owner = world, True
        xs, ys, out_session = rank, (rank - 1) % world, (rank - 2) % world
    else:
        n_sessions, out_owner = world, True
        xs, ys, out_session = rank, rank, rank
    x = _inputs(n, xs, "x", device)
    y = _inputs(n, ys, "y", device)

    gather_mode = "none" if args.no_gather or n_sessions == 1 else args.gather
    owners = [3 * s + 2 for s in range(n_sessions)] if layout == "spmd" else list(range(world))
    root = owners[0]
    gather_bufs, gather_group, pending = None, None, []
    if gather_mode != "none":
        # every session's revealed output, concatenated along rows.  Double-buffered:
        # step k's transfer runs on the RCCL stream while step k+1 computes.
        if gather_mode == "all" or rank == root:
            gather_bufs = [torch.empty((n_sessions * n, n), dtype=torch.float64, device=device)
                           for _ in range(2)]
        if gather_mode == "all" and layout == "spmd":  # the output owners of every session
            gather_group = dist.new_group(owners)

    if layout == "spmd":
        from moose_amd.parallel.spmd import SPMDSession
        from moose_amd.parallel.transport import Transport

        roles = {r: 3 * (rank // 3) + i for i, r in enumerate(ROLES)}
        transport = comm = Transport(rank, world, device)

        def new_session():
            return SPMDSession(ROLES[rank % 3], roles, transport, device)
    elif layout == "cyclic":
        from moose_amd.parallel.cyclic import CyclicSession
        from moose_amd.parallel.cyclic import RingComm
        from moose_amd.parallel.cyclic import default_offsets

        comm = RingComm(rank, world, device)
        offsets = default_offsets(ROLES)

        def new_session():
            return CyclicSession(comm, offsets, device)
    else:
        def new_session():
            return StackedSession(device)

    if layout == "stacked":
        comm = None
    n_steps = [0]
    # MOOSEX_BENCH_STREAMS=n (stacked layout): consecutive steps alternate between n HIP
    # streams so one step's VALU-bound kernels could overlap the previous step's GEMM (the
    # GEMM scratch is per stream).  Measured: 16.6 ms/step with 1 stream, 17.1 with 2, 19.1
    # with 3 -- the GEMM keeps the MFMA pipes ~80 % busy and loses clock and CU slots to the
    # overlapping kernels -- so the default is 1.
    nstreams = int(os.environ.get("MOOSEX_BENCH_STREAMS", "1"))
    streams = ([torch.cuda.Stream(device) for _ in range(nstreams)]
               if layout == "stacked" and device.type == "cuda" and nstreams > 1 else None)

    def step():
        if streams is None:
            return _step()
        with torch.cuda.stream(streams[n_steps[0] % len(streams)]):
            return _step()

    def _step():
        sess = new_session()
        interp = Interpreter(sess, {}, fixedpoint_ring=args.ring)
        outs = interp.run(comp, {"x": x, "y": y})
        z = outs["output_0"].v.v if out_owner else None
        if gather_mode != "none" and out_owner:
            while len(pending) >= 2 * max(1, len(owners) - 1):
                pending.pop(0).wait()
            zc = z.contiguous()
            if gather_mode == "all":
                buf = gather_bufs[n_steps[0] % 2]
                pending.append(dist.all_gather_into_tensor(buf, zc, group=gather_group,
                                                           async_op=True))
            elif rank == root:
                buf = gather_bufs[n_steps[0] % 2]
                ops = [dist.P2POp(dist.irecv, buf[i * n:(i + 1) * n], r)
                       for i, r in enumerate(owners) if r != root]
                buf[owners.index(root) * n:(owners.index(root) + 1) * n].copy_(zc)
                pending.extend(dist.batch_isend_irecv(ops))
            else:
                pending.extend(dist.batch_isend_irecv([dist.P2POp(dist.isend, zc, root)]))
        n_steps[0] += 1
        return z

    def drain():
        while pending:
            pending.pop(0).wait()

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    for i in range(args.warmup):
        step()
        if i == 0:  # the first step fills the shared constant caches: let it finish alone
            sync()
    drain()
    sync()
    comm0 = (comm.bytes_sent, comm.messages) if comm is not None else (0, 0)
    # per-step device time: one event pair per step on the issuing stream (no host sync
    # inside the timed loop; read after the final synchronize)
    evs = ([(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for _ in range(args.steps)] if device.type == "cuda" else None)
    t0 = time.perf_counter()
    for i in range(args.steps):
        if evs is not None:
            evs[i][0].record()
        z = step()
        if evs is not None:
            evs[i][1].record()
    drain()  # every step's gather is complete inside the timed region
    sync()
    elapsed = time.perf_counter() - t0
    step_ms = sorted(a.elapsed_time(b) for a, b in evs) if evs is not None else []
    p2p = ((comm.bytes_sent - comm0[0]) / args.steps, (comm.messages - comm0[1]) / args.steps) \
        if comm is not None else (0, 0)
    per_rank = [elapsed]
    if world > 1:
        tdev = device if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        allt = torch.empty(world, dtype=torch.float64, device=tdev)
        dist.all_gather_into_tensor(allt, t)
        per_rank = allt.cpu().tolist()
    elapsed = max(per_rank)
    ms_per_step = elapsed / args.steps * 1e3
    value = n_sessions * n * n * args.steps / elapsed

    check = None
    if args.check and out_owner:
        ref = _inputs(n, out_session, "x", device) @ _inputs(n, out_session, "y", device)
        check = {"max_abs_err": (z - ref).abs().max().item()}
    if args.check and gather_bufs is not None and (gather_mode == "all" or rank == root):
        # the last step's collected outputs: rank r's revealed output is session s(r)'s
        buf = gather_bufs[(n_steps[0] - 1) % 2]
        sess_of = {"cyclic": lambda r: (r - 2) % world, "spmd": lambda r: r // 3,
                   "stacked": lambda r: r}[layout]
        gerr = 0.0
        for i, r in enumerate(owners):
            s_ = sess_of(r)
            ref = _inputs(n, s_, "x", device) @ _inputs(n, s_, "y", device)
            gerr = max(gerr, (buf[i * n:(i + 1) * n] - ref).abs().max().item())
        check = dict(check or {}, gathered_max_abs_err=gerr)
    checks = [check]
    if world > 1 and args.check:
        checks = [None] * world
        dist.all_gather_object(checks, check)

    if rank == 0:
        parallelism = {
            "stacked": f"dp{world} (one stacked 3-party session per GPU, no inter-GPU reshare)",
            "cyclic": (f"{n_sessions} 3-party sessions on {world} GPUs, each party on its own "
                       "GPU (cyclic layout): every reshare an RCCL send/recv" if world > 1 else
                       "1 stacked 3-party session"),
            "spmd": f"dp{n_sessions} x 3-party sessions, one party per GPU (RCCL reshare)",
        }[layout]
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
            "dtype": f"fixed(14,23) over Z_2^{args.ring} (exact multi-modular int8-MFMA GEMM)",
            "data": "synthetic uniform[-4,4) inputs, device resident",
            "config": {
                "model": f"replicated fixed(14,23) RingDot {n}x{n} (share+dot+trunc_pr+reveal)",
                "global_batch": n_sessions,
                "seq_len": n,
                "parallelism": parallelism,
            },
            "layout": layout,
            "step_streams": len(streams) if streams is not None else 1,
            "gather": gather_mode,
            "world_size": world,
            "sessions": n_sessions,
            "per_rank_ms_per_step": [t / args.steps * 1e3 for t in per_rank],
            # rank 0's point-to-point traffic (inter-party shares over RCCL/xGMI) per step
            "p2p_bytes_per_step_rank0": p2p[0],
            "p2p_messages_per_step_rank0": p2p[1],
        }
        if step_ms:
            line["step_ms_rank0"] = {"min": step_ms[0], "median": step_ms[len(step_ms) // 2],
                                     "max": step_ms[-1]}
        line["device"] = _device_info(device)
        line["revision"] = _revision()
        if args.check:
            line["check"] = [c for c in checks if c is not None]
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
