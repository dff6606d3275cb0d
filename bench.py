#!/usr/bin/env python
"""Headline benchmark: replicated fixed-point matrix product throughput, plus private
logistic-regression inference latency (the two halves of BASELINE.json's metric).

Matmul (the JSON line's ``value``) -- one step is the reference's dot benchmark
(``benchmarks/pymoose/dot_product.py``) at the BASELINE config 3 size: x (alice) and y (bob)
are cast to fixed(14,23), secret-shared onto a 3-party replicated placement, multiplied
(RSS dot = exact multi-modular int8-MFMA GEMM + zero share + reshare), truncated (TruncPr)
and revealed to carole, who decodes to float64.  As in pymoose every fixed dtype runs over
Z_2^128 (``--ring 64`` selects the Z_2^64 path).  Value = output elements per second over
the whole job (all GPUs).

LR inference (``lr_inference`` in the line) -- the reference's ml-inference-with-onnx
tutorial model (``moose_amd/models/predictors/tutorial.py``: 200 x 10 rows, fixed(24,40),
Z_2^128, secure sigmoid) through ``predictors.from_onnx``: p50 latency of whole
evaluations (share -> predict -> reveal) on rank 0's GPU, eager and hipGraph replay, and
with >= 3 GPUs also one party per GPU (SPMD over RCCL).  Measured after the timed matmul
steps, outside their timed region.

Layouts (``--layout``; default ``auto`` = stacked on 1 and 2 GPUs, cyclic on N >= 3: with
two GPUs the three parties of a session cannot sit on three different GPUs, so the cyclic
layout would only add xGMI traffic -- 8.5 share-tensor units per GPU and step on its one
link -- without separating the parties):

* ``stacked`` -- one 3-party session per GPU, all three parties' local work batched into
  one kernel per protocol step; N GPUs = N data-parallel session replicas.
* ``cyclic`` -- N sessions on N GPUs, every party of a session on a DIFFERENT GPU (role r
  of session s on GPU (s + r) mod N, ``moose_amd/parallel/cyclic.py``): each GPU does one
  session's worth of work and every reshare / dealer message / reveal is an RCCL
  send/recv over xGMI.  Weak scaling with the same per-GPU work as the 1-GPU stacked run.
* ``spmd`` -- one party per GPU, N/3 sessions (latency layout).

``--step-streams S``: consecutive steps (independent sessions) alternate between S HIP
streams, each with its own RCCL communicator, so one step's exchanges overlap the next
step's GEMM (the reference runs independent operations as concurrent tasks).  Default 2 for
the cyclic layout at N > 1, else 1.

With several sessions, the revealed outputs of every session are collected on rank 0 (the
client, as the reference's benchmark collects them) over RCCL inside the timed region,
overlapped with the next step (``--gather all`` all-gathers them to every rank instead).
Inputs are synthetic (uniform [-4, 4)), device-resident; tracing/conversion happens once
before the timed region (the reference's client-side compile).  Every step creates a fresh
session (fresh PRF keys).  After the timed steps the last step's outputs are checked
against float64 torch on every rank (``--no-check`` skips it).

Failing loudly (``moose_amd/utils/benchwatch.py``): the whole run has one wall-clock
deadline (``--deadline``, default 540 s, under the driver's 600 s).  Every phase (init +
rendezvous, preflight, warmup, timed, then the optional extras) runs under a watchdog budget
clipped to it; an extra is skipped (and listed) when too little time is left; ``phase_s``
in the line records what each phase took.  Before the warmup every rank does one grouped
round trip with each of its peers on every communicator it will use and verifies who
answered.

Launch: ``python bench.py --gpus N`` starts torch.distributed.run on 127.0.0.1 itself.
Under a launcher (WORLD_SIZE set) each rank process is a supervisor that never touches the
GPU: it runs the rank's worker as a child process, and the supervisors walk a fallback
ladder together -- an attempt that fails or stalls before its headline is killed on every
rank and a fresh one starts (cyclic with 2 step streams -> 1 step stream -> stacked over
gloo); ``attempts`` in the line says which configuration produced the number.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

_T_START = time.monotonic()  # "init" in phase_s counts the imports too

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

REFERENCE_ELEMS_PER_SEC = 1.0e6 / 5.910  # benchmarks/README.md:21, 1000x1000 Fixed128
ROLES = ("alice", "bob", "carole")
METRIC = "replicated fixed(14,23) matmul elems/sec"


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
    ap.add_argument("--link-probe-mib", type=int, default=256,
                    help="after the headline (cyclic, N > 1): point-to-point GB/s of the "
                         "layout's exchange pattern with this many MiB per message (0: off)")
    ap.add_argument("--spmd-configs", action=argparse.BooleanOptionalAction, default=True,
                    help="with >= 3 GPUs also time BASELINE configs 2 (tutorials/"
                         "dotprod.moose) and 3 (RingDot, one party per GPU) on ranks 0-2")
    ap.add_argument("--zero-slot-steps", type=int, default=10,
                    help="one GPU, stacked: also time this many steps with the opt-in "
                         "zero-slot-aware product (reported apart from the headline)")
    ap.add_argument("--ring", type=int, default=128, choices=[64, 128])
    ap.add_argument("--gather", default="root", choices=["root", "all", "none"],
                    help="revealed outputs of every session: to rank 0 (the client; "
                         "default), all-gathered to every rank, or left on their owners")
    ap.add_argument("--no-gather", action="store_true", help="= --gather none")
    ap.add_argument("--layout", default="auto", choices=["auto", "stacked", "cyclic", "spmd"])
    ap.add_argument("--step-streams", type=int, default=None,
                    help="HIP streams (and RCCL communicators) consecutive steps alternate "
                         "between (default: 2 for cyclic at N > 1, else 1)")
    ap.add_argument("--check", dest="check", action="store_true", default=True,
                    help="verify the last step's outputs against float64 torch (default)")
    ap.add_argument("--no-check", dest="check", action="store_false")
    ap.add_argument("--lr-runs", type=int, default=30,
                    help="LR-inference evaluations per mode (0 = skip)")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="process-group backend (auto: RCCL on GPUs, gloo on the CPU and "
                         "with MOOSEX_SHARED_GPU=1)")
    ap.add_argument("--deadline", type=float, default=float(os.environ.get(
        "MOOSEX_BENCH_DEADLINE", "540")),
        help="wall-clock seconds for the whole run (every phase budget is carved out of "
             "it; the driver's own limit is 600 s)")
    return ap.parse_args()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _base_line(args, world):
    """The fields of the JSON line that do not depend on the measurement."""
    return {"metric": METRIC, "value": None, "unit": "output elems/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
            "scaling": "weak", "dtype": f"fixed(14,23) over Z_2^{args.ring}",
            "data": "synthetic uniform[-4,4) inputs, device resident",
            "config": {"model": f"replicated fixed(14,23) RingDot {args.size}x{args.size} "
                                "(share+dot+trunc_pr+reveal)",
                       "seq_len": args.size}}


def _benchwatch():
    """The watchdog/supervisor module, loaded by path: importing the moose_amd package would
    pull in torch and the native libraries, and the supervising processes must stay away
    from the GPU."""
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "moosex_benchwatch", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                          "moose_amd", "utils", "benchwatch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _self_launch(args):
    """N > 1 without a launcher: start the launcher (N rank supervisors, each of which runs
    its rank's worker as a child) under a wall-clock limit of the deadline plus a grace.
    This process never touches the GPU (only argparse ran), and exits with the launcher's
    status (or 3 with an error line if the rank group hangs)."""
    benchwatch = _benchwatch()
    rdir = os.environ.get("MOOSEX_BENCH_RUN_DIR") or tempfile.mkdtemp(prefix="moosex_bench_")
    os.makedirs(rdir, exist_ok=True)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["MOOSEX_BENCH_RUN_DIR"] = rdir
    return benchwatch.supervise(cmd, env, args.gpus, args.deadline + 45,
                                _base_line(args, args.gpus), rdir)


def _resolve(args, world):
    """(layout, step streams, backend) the run will use."""
    layout = args.layout
    if layout == "auto":
        layout = "stacked" if world < 3 else "cyclic"
    nstreams = args.step_streams
    if nstreams is None:
        # cyclic at N > 1: two steps in flight.  A step's dependency chain is its compute
        # plus four message rounds (share, tail A, tail B, reveal: ~4-5 ms each for a
        # 268 MB share tensor on one xGMI link), about twice its compute.  A third stream
        # would cover a slower link, but three steps computing at once cost 4.5 % on the
        # GPU (one GPU, no messages: 16.33 ms with 2 streams, 17.08 ms with 3)
        nstreams = int(os.environ.get("MOOSEX_BENCH_STREAMS",
                                      "2" if layout == "cyclic" and world > 1 else "1"))
    backend = args.backend
    if backend == "auto":
        gpu = os.environ.get("MOOSEX_SHARED_GPU") != "1" and _has_gpus()
        backend = "nccl" if gpu else "gloo"
    return layout, max(1, nstreams), backend


def _has_gpus():
    """Whether a GPU is present, asked without torch (a supervisor never imports it): the
    ROCm kernel driver's device node.  Only labels the supervisor's rungs; the worker
    decides with ``torch.cuda.is_available()``."""
    return os.path.exists("/dev/kfd") and os.environ.get("HIP_VISIBLE_DEVICES", "x") != ""


def _ladder(args, world):
    """The fallback rungs under a launcher: the requested configuration, then (cyclic with
    several step streams) one step stream, then the stacked layout over gloo with no
    inter-GPU traffic at all.  ``reserve_s``: what a rung needs at least (at the default
    deadline); earlier rungs must measure their headline before the later ones' reserve."""
    layout, nstreams, backend = _resolve(args, world)
    base = list(sys.argv[1:])
    rungs = [{"argv": base, "reserve_s": 120,
              "label": {"layout": layout, "streams": nstreams, "backend": backend}}]
    if layout == "cyclic" and nstreams > 1:
        rungs.append({"argv": base + ["--step-streams", "1"], "reserve_s": 150,
                      "label": {"layout": layout, "streams": 1, "backend": backend}})
    if not (layout == "stacked" and backend == "gloo"):
        rungs.append({"argv": base + ["--layout", "stacked", "--gather", "none",
                                      "--backend", "gloo", "--step-streams", "1",
                                      "--no-spmd-configs", "--link-probe-mib", "0"],
                      "reserve_s": 75,
                      "label": {"layout": "stacked", "streams": 1, "backend": "gloo"}})
    return rungs


def _inputs(n, session, which, device):
    import torch

    g = torch.Generator(device="cpu").manual_seed(1234 + 2 * session + (which == "y"))
    return (torch.rand(n, n, generator=g, dtype=torch.float64) * 8 - 4).to(device)


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
    # communication/runtime knobs in effect (RCCL reads the NCCL_* names)
    info["env"] = {k: v for k, v in sorted(os.environ.items())
                   if k.startswith(("NCCL_", "RCCL_", "HSA_", "GPU_MAX_HW_QUEUES", "HIP_"))}
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


# ---------------------------------------------------------------------------------------
# preflight: one grouped round trip with every peer on every communicator
# ---------------------------------------------------------------------------------------
def _link_probe(comm, world, rank, device, prog, dists, mib, reps=3):
    """Point-to-point bandwidth of the layout's exchange pattern, after the headline: every
    rank sends ``mib`` MiB to rank + d and receives as much from rank - d (one grouped
    exchange), for each distance d the cyclic layout uses, then for all of them at once
    (the step's pattern).  GB/s per rank and direction = bytes / the slowest rank's best
    time of ``reps``.  Gives the xGMI/RCCL numbers the step's link model needs."""
    import torch
    import torch.distributed as dist

    nccl = dist.get_backend() == "nccl"
    tdev = device if nccl else torch.device("cpu")
    bdev = [device.index] if device.type == "cuda" and nccl else None
    nbytes = mib << 20
    src = torch.full((nbytes // 8,), rank, dtype=torch.int64, device=device)

    def timed(ds, tick):
        bufs = [torch.empty_like(src) for _ in ds]
        best = float("inf")
        for r in range(reps + 1):
            prog.tick(tick)
            dist.barrier(device_ids=bdev)
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            comm.exchange([(src, (rank + d) % world) for d in ds],
                          [(b, (rank - d) % world) for b, d in zip(bufs, ds)])
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            if r:  # the first round warms the connections up
                best = min(best, time.perf_counter() - t0)
        for b, d in zip(bufs, ds):
            if int(b[0].item()) != (rank - d) % world:
                raise RuntimeError(f"link probe: wrong payload from rank {(rank - d) % world}")
        t = torch.tensor([best], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return round(len(ds) * nbytes / t.item() / 1e9, 2)

    def latency(d, nb, tick, reps=25):
        """Median time of ONE grouped exchange of ``nb`` bytes to rank + d / from rank - d
        (the shape of one protocol round), synchronised on both sides; max over ranks."""
        s = torch.full((max(1, nb // 8),), rank, dtype=torch.int64, device=device)
        b = torch.empty_like(s)
        ts = []
        for r in range(reps + 2):
            prog.tick(tick)
            dist.barrier(device_ids=bdev)
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            comm.exchange([(s, (rank + d) % world)], [(b, (rank - d) % world)])
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            if r >= 2:
                ts.append(time.perf_counter() - t0)
        ts.sort()
        t = torch.tensor([ts[len(ts) // 2]], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return round(t.item() * 1e6, 1)

    rec = {"mib": mib, "reps": reps, "backend": dist.get_backend(),
           "gbs_per_rank_and_direction": {}, "exchange_latency_us_p50": {}}
    for i, d in enumerate(dists):
        rec["gbs_per_rank_and_direction"][f"d{d}"] = timed([d], i)
    rec["gbs_per_rank_and_direction"]["all"] = timed(list(dists), len(dists))
    # small messages: the LR inference's rounds carry 2-4 KB per message
    for i, d in enumerate(dists):
        for nb in (8, 4096, 65536):
            rec["exchange_latency_us_p50"][f"d{d}_{nb}B"] = latency(d, nb, 100 + i)
    return rec


def _preflight(layout, comms, world, rank, device, prog, offsets=None):
    """Each rank sends its rank id to every peer it will exchange with and checks what it
    receives (catches a wrong peer map, a dead link or an RCCL set-up hang before the
    measured work starts).  Returns a short record for the JSON line."""
    import torch
    import torch.distributed as dist

    t0 = time.perf_counter()
    tdev = device if world > 1 and dist.get_backend() == "nccl" else torch.device("cpu")
    if world > 1:
        prog.tick(0)
        one = torch.ones(1, dtype=torch.float64, device=tdev)
        dist.all_reduce(one)
        if int(one.item()) != world:
            raise RuntimeError(f"preflight all_reduce gave {one.item()} on {world} ranks")
    peers = []
    if layout == "cyclic" and world > 1:
        off = list(offsets.values())
        dists = sorted({(b - a) % world for a in off for b in off} - {0})
        for k, comm in enumerate(comms):
            prog.tick(1 + k)
            sends, recvs, expect = [], [], []
            for d in dists:
                src = (rank - d) % world
                buf = torch.full((4,), -1, dtype=torch.int64, device=device)
                sends.append((torch.full((4,), rank, dtype=torch.int64, device=device),
                              (rank + d) % world))
                recvs.append((buf, src))
                expect.append(src)
            comm.exchange(sends, recvs)
            got = [int(b[0].item()) for b, _ in recvs]
            if got != expect:
                raise RuntimeError(f"preflight: rank {rank} expected peers {expect}, got {got}")
            peers = sorted(set(expect) | {(rank + d) % world for d in dists})
    elif layout == "spmd" and world >= 3:
        base = 3 * (rank // 3)
        others = [base + i for i in range(3) if base + i != rank]
        tr = comms[0]
        prog.tick(1)
        bufs = [torch.full((4,), -1, dtype=torch.int64, device=device) for _ in others]
        tr.exchange([(torch.full((4,), rank, dtype=torch.int64, device=device), o)
                     for o in others], list(zip(bufs, others)))
        got = [int(b[0].item()) for b in bufs]
        if got != others:
            raise RuntimeError(f"preflight: rank {rank} expected {others}, got {got}")
        peers = others
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    return {"ok": True, "peers_rank0": peers, "ms": round((time.perf_counter() - t0) * 1e3, 2)}


# ---------------------------------------------------------------------------------------
# LR inference (BASELINE config 4)
# ---------------------------------------------------------------------------------------
def _lr_stacked(runs, device, world=1):
    """p50 latency of the tutorial model on one GPU: eager, then hipGraph replay; then the
    three parties as threads of this process on three streams of this GPU ("parties") and,
    in a run with >= 3 GPUs, on three GPUs ("parties_3gpu": every message a peer copy over
    xGMI)."""
    import numpy as np
    import torch

    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.runtime.local import LocalMooseRuntime

    tm = logistic_regression_tutorial(128)
    out = {}
    # eager (use_graphs=False), replay from the first evaluation (True), the runtime's
    # default with no flags (auto: captured at the second evaluation, replayed after), and
    # the three parties as threads of this process, each on its own HIP stream
    # (parallel/threads.py; per-party tapes replayed by one host thread)
    # "storage" / "parties_storage": the same model with x read from alice's storage (a
    # Load; replayed through runtime/storage_tap.py), runtime defaults
    modes = ["eager", "graphs", "default", "storage", "parties", "parties_storage"]
    gpus3 = None
    if (device.type == "cuda" and world >= 3 and torch.cuda.device_count() >= 3
            and os.environ.get("MOOSEX_SHARED_GPU") != "1"):
        gpus3 = [device] + [torch.device("cuda", (device.index + k) % torch.cuda.device_count())
                            for k in (1, 2)]
        modes.append("parties_3gpu")
    for mode in modes:
        flags = {"eager": {"use_graphs": False}, "graphs": {"use_graphs": True},
                 "default": {}, "storage": {},
                 "parties": {"device_map": {r: str(device) for r in ROLES}, "timeout": 30},
                 "parties_storage": {"device_map": {r: str(device) for r in ROLES},
                                     "timeout": 30},
                 "parties_3gpu": {"device_map": {r: str(d) for r, d in zip(ROLES, gpus3 or [])},
                                  "timeout": 30},
                 }[mode]
        try:
            rt = LocalMooseRuntime(list(ROLES), device=device, fixedpoint_ring=128, **flags)
            comp, args = tm.computation, {"x": tm.x_test}
            if mode.endswith("storage"):
                comp, args = _storage_fed_lr(tm, rt)
            for _ in range(3):
                r = rt.evaluate_computation(comp, args)
            lat = []
            for _ in range(runs):
                t0 = time.perf_counter()
                r = rt.evaluate_computation(comp, args)  # synchronises the device
                lat.append((time.perf_counter() - t0) * 1e3)
        except Exception as e:  # noqa: BLE001 - an extra mode: record, keep the others
            if not (mode.startswith("parties") or mode.endswith("storage")):
                raise
            out[mode] = {"error": f"{type(e).__name__}: {e}"[:300]}
            continue
        err = float(np.abs(np.asarray(list(r.values())[0]) - tm.proba).max())
        lat.sort()
        rec = {"p50_ms": lat[len(lat) // 2], "p90_ms": lat[int(0.9 * (len(lat) - 1))],
               "max_abs_err_vs_sklearn": err}
        if mode.startswith("parties"):
            tapes = [t for _, t in rt._party_tapes.values() if t]
            rec["replayed"] = bool(tapes)
            rec["rounds"] = rt.last_stats.rounds
            if tapes:
                iss = sorted(tapes[0].issue_s)
                rec["host_issue_ms_p50"] = iss[len(iss) // 2] * 1e3
                # one composed graph (one GPU), per-party graphs with device-side message
                # flags (several GPUs), or per-action issue (the fallback)
                rec["replay_form"] = tapes[0].replay_form
                # per-party graphs are checked at capture against the per-action replay
                # (bitwise); a failure keeps the per-action replay and is recorded here
                rec["validated"] = tapes[0].validated
                if tapes[0].fallback:
                    rec["fallback"] = tapes[0].fallback[:200]
        elif mode != "eager":
            rec["captured"] = bool(rt._graphs.plans)
        out[mode] = rec
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if (mode == "parties_3gpu" and rec.get("replay_form") == "party_graphs"
                and not err < 1e-4 and os.environ.get("MOOSEX_PARTY_STREAMS") is None):
            # the per-party graphs' peer pushes delivered wrong data on this node: measure the
            # per-action replay too (its messages are stream-ordered peer copies), so the
            # line still has a valid three-GPU number, and keep both records
            os.environ["MOOSEX_PARTY_STREAMS"] = "0"
            try:
                alt = _lr_stacked_mode(tm, device, flags, runs)
            finally:
                os.environ.pop("MOOSEX_PARTY_STREAMS", None)
            out["parties_3gpu_per_action"] = alt
    return out


def _storage_fed_lr(tm, rt):
    """The tutorial model with its input Loaded from alice's storage (the reference's
    storage-fed worker deployment): (computation, arguments) and x written to storage."""
    from moose_amd.runtime import storage_tap
    from moose_amd.runtime.local import to_native

    native = to_native(tm.computation, 128)
    inputs = [op for op in native.operations if op.kind == "Input"]
    names = {op.attrs.get("arg_name") or op.name for op in inputs}
    for op in inputs:
        rt.write_value_to_storage(op.placement.owner, op.attrs.get("arg_name") or op.name,
                                  tm.x_test)
    return storage_tap.storage_fed(native, names), {}


def _lr_stacked_mode(tm, device, flags, runs):
    """One extra LR parties measurement (bench fallback): p50 / p90 / error / replay form."""
    import numpy as np

    from moose_amd.runtime.local import LocalMooseRuntime

    try:
        rt = LocalMooseRuntime(list(ROLES), device=device, fixedpoint_ring=128, **flags)
        args = {"x": tm.x_test}
        for _ in range(3):
            r = rt.evaluate_computation(tm.computation, args)
        lat = []
        for _ in range(runs):
            t0 = time.perf_counter()
            r = rt.evaluate_computation(tm.computation, args)
            lat.append((time.perf_counter() - t0) * 1e3)
    except Exception as e:  # noqa: BLE001 - an extra record
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    lat.sort()
    tapes = [t for _, t in rt._party_tapes.values() if t]
    return {"p50_ms": lat[len(lat) // 2], "p90_ms": lat[int(0.9 * (len(lat) - 1))],
            "max_abs_err_vs_sklearn": float(np.abs(np.asarray(list(r.values())[0])
                                                   - tm.proba).max()),
            "replay_form": tapes[0].replay_form if tapes else None,
            "validated": tapes[0].validated if tapes else None, "rounds": rt.last_stats.rounds}


def _lr_spmd(runs, world, rank, device, prog):
    os.environ.setdefault("MOOSEX_TAPE_TIMING", "1")  # per-round device time in the record
    """The tutorial model with one party per GPU (ranks 3s, 3s+1, 3s+2 = alice, bob,
    carole of session s): every reshare, dealer message and reveal an RCCL send/recv.
    Latency of an evaluation = max over its three ranks; p50 over ``runs``.  Two modes:
    eager (every op dispatched from Python) and the SPMD tape (parallel/spmd_graphs.py:
    captured kernel segments + prebuilt message rounds, replayed from the third
    evaluation on), with the message rounds per evaluation and the host time a replay
    spends issuing work."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.parallel import spmd_graphs
    from moose_amd.parallel.spmd import SPMDSession
    from moose_amd.parallel.transport import Transport
    from moose_amd.runtime.interpreter import Interpreter
    from moose_amd.runtime.local import to_native

    triples = [list(range(3 * s, 3 * s + 3)) for s in range(world // 3)]
    groups = [dist.new_group(t) for t in triples]  # every rank creates every group
    mine = rank // 3 if rank < 3 * len(triples) else None
    rec = None
    if mine is not None:
        g = groups[mine]
        tm = logistic_regression_tutorial(128)
        comp = to_native(tm.computation, 128)
        # the session's own group: the tape's collective capture decision (spmd_graphs
        # ._agree) must involve these three ranks only (ranks outside every triple, and
        # the other triples, are not in this evaluation)
        tr = Transport(rank, world, device, group=g, plans=True)  # every rank: every argument
        roles = {r: 3 * mine + i for i, r in enumerate(ROLES)}
        me = ROLES[rank % 3]
        bdev = [device.index] if device.type == "cuda" and dist.get_backend() == "nccl" else None
        tdev = device if dist.get_backend() == "nccl" else torch.device("cpu")
        rec = {"ranks": triples[mine]}

        def eager():
            sess = SPMDSession(me, roles, tr, device)
            interp = Interpreter(sess, {}, fixedpoint_ring=128)
            outs = interp.run(comp, {"x": tm.x_test})
            return {k: interp.to_numpy(v) for k, v in outs.items() if sess.materialized(v.v)}, \
                sess.stats

        modes = ("eager", "tape") if spmd_graphs.enabled(device) else ("eager",)
        for mode in modes:
            lat, tape, got, stats = [], None, None, None
            for i in range(runs + 3):
                prog.tick(i)
                dist.barrier(group=g, device_ids=bdev)
                t0 = time.perf_counter()
                r = None
                if mode == "tape":
                    r = spmd_graphs.evaluate(comp, {"x": tm.x_test}, me, roles, tr, device, {},
                                             128)
                if r is None:
                    got, stats = eager()
                else:
                    got, stats, tape = r
                if device.type == "cuda":
                    torch.cuda.synchronize(device)
                if i >= 3:
                    lat.append((time.perf_counter() - t0) * 1e3)
            mine_t = torch.tensor(lat, dtype=torch.float64, device=tdev)
            allt = torch.empty(3 * runs, dtype=torch.float64, device=tdev)
            dist.all_gather_into_tensor(allt, mine_t, group=g)
            per_run = allt.reshape(3, runs).max(dim=0).values.cpu().numpy()
            per_run.sort()
            m = {"p50_ms": float(per_run[len(per_run) // 2]),
                 "p90_ms": float(per_run[int(0.9 * (runs - 1))]), "rounds": stats.rounds}
            if mode == "tape":
                m["replayed"] = tape is not None and tape.replays >= runs
                if tape is not None and tape.issue_s:
                    med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731
                    m["host_issue_ms_p50"] = med(tape.issue_s) * 1e3
                    m["tape_rounds"], m["tape_segments"] = tape.rounds, tape.segments
                    # where a replay's time goes: host time inside the message rounds, and
                    # (timed replays) the tape stream's time in them -- all rounds and the
                    # longest -- so p50 ~ rounds x per-round latency + kernel time checks out
                    m["comm_host_ms_p50"] = med(tape.comm_host_s) * 1e3
                    if tape.round_device_ms:
                        m["rounds_device_ms_p50"] = med(tape.round_device_ms)
                        m["round_device_max_ms_p50"] = med(tape.round_device_max_ms)
                        m["per_round_device_us"] = med(tape.round_device_ms) * 1e3 / max(
                            1, tape.rounds)
            if rank % 3 == 1:  # bob holds the opened probabilities
                m["max_abs_err_vs_sklearn"] = float(
                    np.abs(np.asarray(list(got.values())[0]) - tm.proba).max())
            rec[mode] = m
    return rec


# The reference's tutorials/dotprod.moose (BASELINE config 2), verbatim: a fixed(24,40)
# 1x3 . 3x1 dot product of two players' constants, revealed to the third.
DOTPROD_MOOSE = """\
constant_0 = Constant{value = HostFloat64Tensor([[1.0, 2.0, 3.0]])}: () -> Tensor<Float64> () @Host(player0)
cast_0 = Cast: (Tensor<Float64>) -> Tensor<Fixed128(24, 40)> (constant_0) @Host(player0)
constant_1 = Constant{value = HostFloat64Tensor([[4.0], [5.0], [6.0]])}: () -> Tensor<Float64> () @Host(player1)
cast_1 = Cast: (Tensor<Float64>) -> Tensor<Fixed128(24, 40)> (constant_1) @Host(player1)
dot_0 = Dot: (Tensor<Fixed128(24, 40)>, Tensor<Fixed128(24, 40)>) -> Tensor<Fixed128(24, 40)> (cast_0, cast_1) @Replicated(player0, player1, player2)
cast_2 = Cast: (Tensor<Fixed128(24, 40)>) -> Tensor<Float64> (dot_0) @Host(player2)
output_0 = Output{tag = "output_0"}: (Tensor<Float64>) -> Tensor<Float64> (cast_2) @Host(player2)
"""


def _spmd_configs(args, world, rank, device, prog):
    """BASELINE configs 2 and 3 on three GPUs (ranks 0, 1, 2, one party each, every
    reshare an RCCL send/recv over xGMI): the reference's tutorials/dotprod.moose latency
    (p50 over ``args.lr_runs`` evaluations) and the headline RingDot at ``args.size`` (ms
    per step over 5 steps).  A step's time is the max over the three ranks."""
    import torch
    import torch.distributed as dist

    from moose_amd.ir import textual
    from moose_amd.parallel.spmd import SPMDSession
    from moose_amd.parallel.transport import Transport
    from moose_amd.runtime.interpreter import Interpreter

    g = dist.new_group([0, 1, 2])  # every rank creates every group
    g6 = dist.new_group(list(range(6))) if world >= 6 else None
    gout = dist.new_group([2, 5]) if world >= 6 else None
    if rank >= 3:
        if world >= 6 and rank < 6:
            return {"config5_dp2_replicas": _config5(args, world, rank, device, prog, g6, gout)}
        return None
    bdev = [device.index] if device.type == "cuda" and dist.get_backend() == "nccl" else None
    tdev = device if dist.get_backend() == "nccl" else torch.device("cpu")
    tr = Transport(rank, world, device, plans=True)

    def timed(comp, roles, args_of, runs, warm):
        lat, outs = [], None
        for i in range(runs + warm):
            prog.tick(i)
            dist.barrier(group=g, device_ids=bdev)
            t0 = time.perf_counter()
            sess = SPMDSession(list(roles)[rank], roles, tr, device)
            outs = Interpreter(sess, {}, fixedpoint_ring=128).run(comp, args_of())
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            if i >= warm:
                lat.append((time.perf_counter() - t0) * 1e3)
        mine = torch.tensor(lat, dtype=torch.float64, device=tdev)
        allt = torch.empty(3 * runs, dtype=torch.float64, device=tdev)
        dist.all_gather_into_tensor(allt, mine, group=g)
        per_run = sorted(allt.reshape(3, runs).max(dim=0).values.cpu().tolist())
        return per_run, outs

    rec = {}
    comp2 = textual.parse_computation(DOTPROD_MOOSE, parallel=False)
    roles2 = {"player0": 0, "player1": 1, "player2": 2}
    runs = max(5, args.lr_runs)
    per, outs = timed(comp2, roles2, dict, runs, 3)
    rec["config2_dotprod_moose"] = {"p50_ms": per[len(per) // 2], "runs": runs}
    if rank == 2:
        got = float(outs["output_0"].v.v.reshape(-1)[0])
        rec["config2_dotprod_moose"]["output"] = got  # 1*4 + 2*5 + 3*6 = 32
    n = args.size
    comp3 = build_computation(args.ring)
    roles3 = {r: i for i, r in enumerate(ROLES)}
    x = _inputs(n, 0, "x", device) if rank == 0 else None
    y = _inputs(n, 0, "y", device) if rank == 1 else None
    feed = lambda: {k: v for k, v in (("x", x), ("y", y)) if v is not None}  # noqa: E731
    per, _ = timed(comp3, roles3, feed, 5, 2)
    ms = sum(per) / len(per)
    rec["config3_ringdot_3gpu"] = {"ms_per_step": ms, "elems_per_sec": n * n / ms * 1e3,
                                   "size": n, "steps": 5}
    if world >= 6:
        rec["config5_dp2_replicas"] = _config5(args, world, rank, device, prog, g6, gout)
    return rec


MPSPDZ_DOT_1000_S = 5.910  # benchmarks/README.md: moose, one 1000x1000 dot, sequential table


def _config5(args, world, rank, device, prog, g6, gout):
    """BASELINE config 5 (benchmarks/mp-spdz parity): two data-parallel replicas of the
    3-party session on six GPUs (ranks 3r, 3r+1, 3r+2 = alice, bob, carole of replica r),
    each step one replicated fixed(14,23) 1000 x 1000 dot per replica -- every reshare an
    RCCL send/recv inside the replica -- and an all-gather of the two revealed outputs
    between the replicas' output owners (ranks 2 and 5).  ms per step = max over the six
    ranks, mean of 5 steps after 2 warmup steps."""
    import torch
    import torch.distributed as dist

    from moose_amd.parallel.spmd import SPMDSession
    from moose_amd.parallel.transport import Transport
    from moose_amd.runtime.interpreter import Interpreter

    rep = rank // 3
    n = min(1000, max(8, args.size // 2))  # the reference's table size (CPU tests: smaller)
    comp = build_computation(args.ring)
    roles = {r: 3 * rep + i for i, r in enumerate(ROLES)}
    # a plan scope of its own: carole holds no argument, so her plan key is the same as in
    # config 3 (other shapes) and must not replay that plan
    tr = Transport(rank, world, device, plans=True, plan_scope="config5")
    x = _inputs(n, rep, "x", device) if rank % 3 == 0 else None
    y = _inputs(n, rep, "y", device) if rank % 3 == 1 else None
    feed = {k: v for k, v in (("x", x), ("y", y)) if v is not None}
    nccl = dist.get_backend() == "nccl"
    bdev = [device.index] if device.type == "cuda" and nccl else None
    gdev = device if nccl else torch.device("cpu")
    both = torch.empty(2 * n * n, dtype=torch.float64, device=gdev)
    lat, steps, warm = [], 5, 2
    for i in range(steps + warm):
        prog.tick(i)
        dist.barrier(group=g6, device_ids=bdev)
        t0 = time.perf_counter()
        outs = Interpreter(SPMDSession(ROLES[rank % 3], roles, tr, device), {},
                           fixedpoint_ring=128).run(comp, feed)
        if rank % 3 == 2:  # the replica's client: collect both replicas' outputs
            z = outs["output_0"].v.v.reshape(-1).to(device=gdev, dtype=torch.float64)
            dist.all_gather_into_tensor(both, z.contiguous(), group=gout)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if i >= warm:
            lat.append((time.perf_counter() - t0) * 1e3)
    err = None
    if rank % 3 == 2:
        err = 0.0
        for r in range(2):
            ref = _inputs(n, r, "x", device) @ _inputs(n, r, "y", device)
            got = both[r * n * n:(r + 1) * n * n].to(device).reshape(n, n)
            err = max(err, (got - ref).abs().max().item())
    t = torch.tensor(lat + [err if err is not None else -1.0], dtype=torch.float64, device=gdev)
    allt = torch.empty(6 * (steps + 1), dtype=torch.float64, device=gdev)
    dist.all_gather_into_tensor(allt, t, group=g6)
    allt = allt.reshape(6, steps + 1).cpu()
    ms = allt[:, :steps].max(dim=0).values.mean().item()
    errs = [e for e in allt[:, steps].tolist() if e >= 0]
    return {"ms_per_step": ms, "replicas": 2, "size": n, "dots_per_step": 2,
            "steps": steps, "dots_per_sec": 2e3 / ms,
            "vs_reference_dots_per_sec": 2e3 / ms * MPSPDZ_DOT_1000_S,
            "gathered_max_abs_err": max(errs) if errs else None}


# ---------------------------------------------------------------------------------------
def main():
    args = _parse()
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if args.gpus > 1 and not world:
        sys.exit(_self_launch(args))
    if world > 1 and os.environ.get("MOOSEX_BENCH_CHILD") != "1":
        # under a launcher: this rank process supervises its worker (a child process) and
        # walks the fallback ladder with the other ranks; it never touches the GPU
        bw = _benchwatch()
        sys.exit(bw.rank_supervisor(os.path.abspath(__file__), int(os.environ["RANK"]), world,
                                    _ladder(args, world), args.deadline,
                                    _base_line(args, world)))
    prog = []
    try:
        _main(args, prog)
    except SystemExit:
        raise
    except BaseException as e:  # noqa: BLE001 - report, then fail
        if prog:
            prog[0].fail(f"{type(e).__name__}: {e}")
            if prog[0].result is not None:
                # the headline was measured and rank 0 reported it with this error noted:
                # an optional extra (LR inference, configs 2/3) failed -- keep it
                os._exit(0)
        raise


def _main(args, prog_out):

    import datetime

    import torch
    import torch.distributed as dist

    from moose_amd.utils.benchwatch import Clock
    from moose_amd.utils.benchwatch import Progress

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started {world} ranks")
    if world > 1:
        # enough HIP hardware queues for the step streams and their RCCL communicators'
        # streams: two streams on one queue serialise (a step's exchange would wait behind
        # the next step's whole GEMM; profiles/r3_stream_concurrency.md).  Read by the HIP
        # runtime when it initialises, i.e. below.
        q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(16, max(q, 8)))
    clock = Clock.from_env(args.deadline)
    prog = Progress(rank, world, clock, lambda: _base_line(args, world),
                    result_path=os.environ.get("MOOSEX_BENCH_RESULT"), t0=_T_START)
    prog_out.append(prog)
    layout, nstreams, backend = _resolve(args, world)
    # MOOSEX_SHARED_GPU=1: every rank on cuda:0 with gloo (rehearsing the multi-GPU
    # layouts on a one-GPU box; RCCL refuses two ranks on one device)
    shared = os.environ.get("MOOSEX_SHARED_GPU") == "1"
    if torch.cuda.is_available():
        idx = 0 if shared else local_rank
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    if device.type != "cuda" or shared:
        backend = "gloo"
    elif args.backend == "auto":
        backend = "nccl"
    if world > 1:
        dist.init_process_group(backend=backend,
                                device_id=device if backend == "nccl" else None,
                                # past the deadline: the watchdog reports first
                                timeout=datetime.timedelta(
                                    seconds=max(60.0, prog.remaining() + 60)))
        prog.phase("rendezvous")
        dist.barrier()

    from moose_amd.runtime.interpreter import Interpreter
    from moose_amd.runtime.session import StackedSession

    if layout == "spmd" and (world < 3 or world % 3):
        raise SystemExit("--layout spmd needs a multiple of 3 GPUs (one per party)")
    nccl = world > 1 and backend == "nccl"
    tdev = device if nccl else torch.device("cpu")

    def fits(name):
        """Every rank agrees whether the optional phase ``name`` still fits the deadline."""
        ok = prog.extra_fits(name)
        if world > 1:
            t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ok = t.item() > 0
        if not ok:
            prog.skip(name)
        return ok

    comp = build_computation(args.ring)
    n = args.size
    if layout == "spmd":
        n_sessions, out_owner = world // 3, rank % 3 == 2
        xs, ys, out_session = rank // 3, rank // 3, rank // 3
    elif layout == "cyclic":  # rank g hosts role r of session g - o(r) (cyclic.py)
        from moose_amd.parallel.cyclic import default_layout

        # link-balanced party offsets and input-share directions for this program
        offsets, share_dirs = default_layout(ROLES, world)
        n_sessions, out_owner = world, True
        xs, ys, out_session = [(rank - offsets[r]) % world for r in ROLES]
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
                           for _ in range(max(2, nstreams))]
        if gather_mode == "all" and layout == "spmd":  # the output owners of every session
            gather_group = dist.new_group(owners)
        elif world > 1 and layout != "spmd":
            # a communicator of its own: on the step streams' communicator the collection of
            # step k would sit in front of step k+2's exchanges (one RCCL stream each)
            gather_group = dist.new_group(list(range(world)))

    streams = ([torch.cuda.Stream(device) for _ in range(nstreams)]
               if device.type == "cuda" and nstreams > 1 else None)
    if layout == "spmd":
        from moose_amd.parallel.spmd import SPMDSession
        from moose_amd.parallel.transport import Transport

        roles = {r: 3 * (rank // 3) + i for i, r in enumerate(ROLES)}
        comms = [Transport(rank, world, device)]

        def new_session(k):
            return SPMDSession(ROLES[rank % 3], roles, comms[0], device)
    elif layout == "cyclic":
        from moose_amd.parallel.cyclic import CyclicSession
        from moose_amd.parallel.cyclic import RingComm

        # one communicator per step stream: RCCL runs the operations of a communicator in
        # issue order, so step k+1's exchanges must not queue behind step k's
        groups = [None] + ([dist.new_group(list(range(world))) for _ in range(nstreams - 1)]
                           if world > 1 else [None] * (nstreams - 1))
        comms = [RingComm(rank, world, device, group=g) for g in groups]

        def new_session(k):
            return CyclicSession(comms[k % len(comms)], offsets, device, share_dirs=share_dirs)
    else:
        comms = []

        def new_session(k):
            return StackedSession(device)

    n_steps = [0]
    gloo_staged = (gather_mode != "none" and device.type == "cuda" and world > 1
                   and dist.get_backend() == "gloo")

    def _gather_staged(zc, k):
        zh = zc.cpu()  # waits for the step's stream
        if gather_mode == "all":
            hb = torch.empty((len(owners) * n, n), dtype=torch.float64)
            dist.all_gather_into_tensor(hb, zh, group=gather_group)
        elif rank == root:
            hb = torch.empty((len(owners) * n, n), dtype=torch.float64)
            ops = [dist.P2POp(dist.irecv, hb[i * n:(i + 1) * n], r, group=gather_group)
                   for i, r in enumerate(owners) if r != root]
            hb[owners.index(root) * n:(owners.index(root) + 1) * n].copy_(zh)
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        else:
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, zh, root,
                                                        group=gather_group)]):
                w.wait()
            return
        gather_bufs[k % len(gather_bufs)].copy_(hb)

    def step():
        if streams is None:
            return _step()
        st = streams[n_steps[0] % len(streams)]
        st.wait_stream(torch.cuda.current_stream(device))  # inputs / previous host work
        with torch.cuda.stream(st):
            return _step()

    def _step():
        k = n_steps[0]
        sess = new_session(k)
        interp = Interpreter(sess, {}, fixedpoint_ring=args.ring)
        outs = interp.run(comp, {"x": x, "y": y})
        z = outs["output_0"].v.v if out_owner else None
        if gather_mode != "none" and out_owner:
            while len(pending) >= 2 * max(1, len(owners) - 1):
                pending.pop(0).wait()
            zc = z.contiguous()
            if gloo_staged:
                # gloo moves host memory: stage the device output through the host, in
                # stream order (one-GPU rehearsals only; RCCL takes the device tensors)
                _gather_staged(zc, k)
            elif gather_mode == "all":
                buf = gather_bufs[k % len(gather_bufs)]
                pending.append(dist.all_gather_into_tensor(buf, zc, group=gather_group,
                                                           async_op=True))
            elif rank == root:
                buf = gather_bufs[k % len(gather_bufs)]
                ops = [dist.P2POp(dist.irecv, buf[i * n:(i + 1) * n], r, group=gather_group)
                       for i, r in enumerate(owners) if r != root]
                buf[owners.index(root) * n:(owners.index(root) + 1) * n].copy_(zc)
                pending.extend(dist.batch_isend_irecv(ops))
            else:
                pending.extend(dist.batch_isend_irecv(
                    [dist.P2POp(dist.isend, zc, root, group=gather_group)]))
        n_steps[0] += 1
        return z

    def drain():
        while pending:
            pending.pop(0).wait()

    def sync():
        if streams is not None:
            cur = torch.cuda.current_stream(device)
            for st in streams:
                cur.wait_stream(st)
        if device.type == "cuda":
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    prog.phase("preflight")
    preflight = _preflight(layout, comms, world, rank, device, prog,
                           offsets if layout == "cyclic" else None)

    prog.phase("warmup")
    for i in range(args.warmup):
        prog.tick(i)
        step()
        if i == 0:  # the first step fills the shared constant caches: let it finish alone
            sync()
    drain()
    sync()
    comm0 = [(c.bytes_sent, c.messages) for c in comms]
    # per-step device time: one event pair per step on the issuing stream (no host sync
    # inside the timed loop; read after the final synchronize)
    evs = ([(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for _ in range(args.steps)] if device.type == "cuda" and streams is None else None)
    prog.phase("timed")
    t0 = time.perf_counter()
    for i in range(args.steps):
        prog.tick(i)
        if evs is not None:
            evs[i][0].record()
        z = step()
        if evs is not None:
            evs[i][1].record()
    drain()  # every step's gather is complete inside the timed region
    sync()
    elapsed = time.perf_counter() - t0
    step_ms = sorted(a.elapsed_time(b) for a, b in evs) if evs is not None else []

    prog.phase("report")
    p2p = [sum(c.bytes_sent for c in comms) - sum(b for b, _ in comm0),
           sum(c.messages for c in comms) - sum(m for _, m in comm0)]
    per_rank = [[elapsed] + p2p]
    if world > 1:
        t = torch.tensor([elapsed] + p2p, dtype=torch.float64, device=tdev)
        allt = torch.empty(3 * world, dtype=torch.float64, device=tdev)
        dist.all_gather_into_tensor(allt, t)
        per_rank = allt.reshape(world, 3).cpu().tolist()
    elapsed = max(r[0] for r in per_rank)
    ms_per_step = elapsed / args.steps * 1e3
    value = n_sessions * n * n * args.steps / elapsed

    parallelism = {
        "stacked": f"dp{world} (one stacked 3-party session per GPU, no inter-GPU reshare"
                   + ("; 3 parties cannot sit on 3 distinct GPUs with 2)" if world == 2 else ")"),
        "cyclic": (f"{n_sessions} 3-party sessions on {world} GPUs, each party on its own "
                   "GPU (cyclic layout): every reshare an RCCL send/recv" if world > 1 else
                   "1 stacked 3-party session"),
        "spmd": f"dp{n_sessions} x 3-party sessions, one party per GPU (RCCL reshare)",
    }[layout]
    line = _base_line(args, world)
    line.update({
        "value": value,
        "ms_per_step": ms_per_step,
        "vs_baseline": value / REFERENCE_ELEMS_PER_SEC,
        "dtype": f"fixed(14,23) over Z_2^{args.ring} (exact multi-modular int8-MFMA GEMM)",
        "layout": layout,
        "step_streams": nstreams,
        "gather": gather_mode,
        "world_size": world,
        "sessions": n_sessions,
        "per_rank_ms_per_step": [r[0] / args.steps * 1e3 for r in per_rank],
        # point-to-point traffic (inter-party shares over RCCL/xGMI) per step and rank
        "p2p_bytes_per_step": [r[1] / args.steps for r in per_rank],
        "p2p_messages_per_step": [r[2] / args.steps for r in per_rank],
        "preflight": preflight,
        "deadline_s": args.deadline,
    })
    line["config"].update(global_batch=n_sessions, parallelism=parallelism)
    if step_ms:
        line["step_ms_rank0"] = {"min": step_ms[0], "median": step_ms[len(step_ms) // 2],
                                 "max": step_ms[-1]}
    line["device"] = _device_info(device)
    if device.type == "cuda":
        # rank 0's device memory: the torch allocator's high-water mark, and what the device
        # reports in use after the steps (this also counts the native GEMM workspaces and
        # the caching allocator's reserve)
        free, total = torch.cuda.mem_get_info(device)
        line["mem_gib_rank0"] = {
            "torch_peak_allocated": round(torch.cuda.max_memory_allocated(device) / 2**30, 2),
            "device_in_use": round((total - free) / 2**30, 2),
            "device_total": round(total / 2**30, 1)}
    line["revision"] = _revision()
    prog.headline_done(line)

    exit_code = 0
    if args.check and fits("check"):
        prog.phase("check")
        check = None
        if out_owner:
            ref = _inputs(n, out_session, "x", device) @ _inputs(n, out_session, "y", device)
            check = {"rank": rank, "max_abs_err": (z - ref).abs().max().item()}
        if gather_bufs is not None and (gather_mode == "all" or rank == root):
            # the last step's collected outputs: rank r's revealed output is session s(r)'s
            buf = gather_bufs[(n_steps[0] - 1) % len(gather_bufs)]
            sess_of = {"cyclic": lambda r: (r - offsets[ROLES[2]]) % world,
                       "spmd": lambda r: r // 3,
                       "stacked": lambda r: r}[layout]
            gerr = 0.0
            for i, r in enumerate(owners):
                s_ = sess_of(r)
                ref = _inputs(n, s_, "x", device) @ _inputs(n, s_, "y", device)
                gerr = max(gerr, (buf[i * n:(i + 1) * n] - ref).abs().max().item())
            check = dict(check or {"rank": rank}, gathered_max_abs_err=gerr)
        checks = [check]
        if world > 1:
            checks = [None] * world
            dist.all_gather_object(checks, check)
        checks = [c for c in checks if c is not None]
        worst = max([c.get("max_abs_err", 0.0) for c in checks]
                    + [c.get("gathered_max_abs_err", 0.0) for c in checks] + [0.0])
        line["check"] = {"ranks": len(checks), "max_abs_err": worst, "ok": worst < 1e-2}
        if worst >= 1e-2:
            line["error"] = f"wrong results: max abs error {worst} vs float64 torch"
            exit_code = 4

    # the optional extras after the headline: each runs only when its expected need is
    # left before the deadline (all ranks agree), under a budget clipped to the deadline;
    # a hang in one fires the watchdog, which reports the measured line with the error
    if layout == "cyclic" and world > 1 and args.link_probe_mib > 0 and fits("link_probe"):
        prog.phase("link_probe")
        off = list(offsets.values())
        dists = sorted({(b - a) % world for a in off for b in off} - {0})
        mib = args.link_probe_mib if dist.get_backend() == "nccl" else 1  # gloo: path only
        probe = _link_probe(comms[0], world, rank, device, prog, dists, mib)
        if rank == 0:
            line["link_probe"] = probe

    if args.lr_runs > 0 and fits("lr"):
        prog.phase("lr")
        lr = {"model": "ml-inference-with-onnx tutorial LogisticRegression (200x10, "
                       "fixed(24,40), Z_2^128, from_onnx)"}
        if rank == 0:
            lr["one_gpu"] = _lr_stacked(args.lr_runs, device, world)
        if world > 1:
            dist.barrier()
        if world >= 3 and args.spmd_configs and fits("lr_spmd"):
            prog.phase("lr_spmd")
            rec = _lr_spmd(args.lr_runs, world, rank, device, prog)
            recs = [None] * world
            dist.all_gather_object(recs, rec)
            mine = [r for r in recs if r is not None and 0 in r.get("ranks", [])]
            if mine:
                r0 = dict(mine[0])
                for mode in ("eager", "tape"):  # bob's accuracy into rank 0's record
                    if mode not in r0:
                        continue
                    errs = [r[mode].get("max_abs_err_vs_sklearn") for r in recs
                            if r is not None and r.get("ranks") == r0["ranks"]
                            and r[mode].get("max_abs_err_vs_sklearn") is not None]
                    r0[mode] = dict(r0[mode], max_abs_err_vs_sklearn=errs[0] if errs else None)
                lr["spmd_one_party_per_gpu"] = r0
        if rank == 0:
            line["lr_inference_p50_ms"] = {k: v["p50_ms"] for k, v in lr["one_gpu"].items()
                                           if "p50_ms" in v}
            sp = lr.get("spmd_one_party_per_gpu")
            if sp:
                # the faster of the replayed tape and eager dispatch (both are in
                # lr_inference.spmd_one_party_per_gpu; "spmd_mode" says which one this is)
                cands = [("eager", sp["eager"])]
                if sp.get("tape", {}).get("replayed"):
                    cands.append(("tape", sp["tape"]))
                mode, best = min(cands, key=lambda kv: kv[1]["p50_ms"])
                line["lr_inference_p50_ms"]["spmd"] = best["p50_ms"]
                line["lr_inference_p50_ms"]["spmd_eager"] = sp["eager"]["p50_ms"]
                if "tape" in sp:
                    line["lr_inference_p50_ms"]["spmd_tape"] = sp["tape"]["p50_ms"]
                line["lr_inference_spmd_mode"] = mode
                line["lr_inference_rounds"] = best["rounds"]
            line["lr_inference"] = lr

    if world >= 3 and args.spmd_configs and fits("spmd_configs"):
        prog.phase("spmd_configs")
        rec = _spmd_configs(args, world, rank, device, prog)
        recs = [None] * world
        dist.all_gather_object(recs, rec)
        if rank == 0:
            merged = dict(recs[0] or {})
            out2 = (recs[2] or {}).get("config2_dotprod_moose", {}).get("output")
            if "config2_dotprod_moose" in merged:
                merged["config2_dotprod_moose"]["output"] = out2
            if "config5_dp2_replicas" in merged:
                line["config5_dp2_replicas"] = merged.pop("config5_dp2_replicas")
            line["spmd_three_gpus"] = merged

    if (world == 1 and layout == "stacked" and args.zero_slot_steps > 0
            and fits("zero_slot")):
        # secondary figure, NOT the headline: the same steps with the zero-slot-aware RSS
        # product (protocols/replicated.py _zero_slot_cross, opt-in MOOSEX_ZERO_SLOTS=1):
        # both operands are fresh input sharings with a public zero slot, so each party's
        # cross product is one K-long GEMM instead of the K-doubled one
        from moose_amd.protocols import replicated as rep_mod

        prog.phase("zero_slot")
        prev, rep_mod.ZERO_SLOTS = rep_mod.ZERO_SLOTS, True
        try:
            for _ in range(2):
                step()
            sync()
            tz = time.perf_counter()
            for _ in range(args.zero_slot_steps):
                zz = step()
            sync()
            zms = (time.perf_counter() - tz) / args.zero_slot_steps * 1e3
            line["zero_slot_aware"] = {
                "ms_per_step": zms, "value": n * n / zms * 1e3, "steps": args.zero_slot_steps,
                # TruncPr rounds probabilistically: ~1 ulp (2^-23) apart
                "max_abs_diff_vs_headline_output": (zz - z).abs().max().item(),
                "note": "opt-in MOOSEX_ZERO_SLOTS=1, not the headline: skips the cross terms "
                        "that multiply a fresh input sharing's public zero slot (half the "
                        "GEMM)"}
        finally:
            rep_mod.ZERO_SLOTS = prev

    prog.phase("done")
    prog.disarm()
    prog.emit(line)
    if world > 1:
        dist.destroy_process_group()
    if exit_code:
        sys.exit(exit_code)


if __name__ == "__main__":
    main()
