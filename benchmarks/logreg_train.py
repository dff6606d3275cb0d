"""Private logistic-regression training benchmark (mini-batch SGD with momentum).

Workload parity with the reference's ``benchmarks/pymoose/logreg.py``: 100 features,
``fixed(24, 40)`` (ring 128), learning rate 0.1, momentum 0.9, one epoch over
``n_iter`` batches of ``batch_size`` rows; the data lives on alice, the initial weights on
bob, ``1/batch_size`` is a mirrored (public, replicated-everywhere) constant, and every
training step runs on the replicated placement.  BASELINE.md quotes the reference's wall
time for (batch_size, n_iter) in {128..2048} x {10, 50, 100} (3 gRPC workers on one
host); this script reports the same quantity for our runtime.

The model is traced once per configuration; the plan is converted to the native IR once
and each experiment is one evaluation of it (the reference likewise reports the workers'
own session time, ``max(timings.values())``).

Usage::

    python benchmarks/logreg_train.py --batch_size 128 --n_iter 10 --n_exp 3 \
        [--runtime local|parties|distributed] [--device cuda|cpu] [--json out.json]

``--runtime parties``: the three parties as threads of this process, each on its own HIP
stream (``--devices``: one device per party, e.g. ``cuda:0,cuda:1,cuda:2``; default all on
``--device``), every reshare / dealer message a device copy between them -- the
per-party protocol the reference's three workers run (parallel/threads.py), instead of
the stacked one-session simulation of ``local``.  With ``--graphs`` the parties' tapes are
replayed as one composed graph (one device) or per-party graphs (several).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import moose_amd as pm  # noqa: E402

N_FEATURES = 100
LEARNING_RATE = 0.1
MOMENTUM = 0.9
FIXED = pm.fixed(24, 40)

# the reference's published moose wall times (seconds), keyed (batch_size, n_iter):
# benchmarks/README.md:44-48 of the reference, as tabulated in BASELINE.md (main table).
# The reference published no batch-256 row.
REFERENCE_S = {
    (128, 10): 1.316, (128, 50): 7.091, (128, 100): 14.385,
    (512, 10): 1.981, (512, 50): 10.134, (512, 100): 20.819,
    (1024, 10): 2.963, (1024, 50): 15.033, (1024, 100): 31.017,
    (2048, 10): 4.730, (2048, 50): 24.266, (2048, 100): 63.100,
}


def build_training(batch_size: int, n_batches: int, n_features: int = N_FEATURES,
                   lr: float = LEARNING_RATE, momentum: float = MOMENTUM, fixed=FIXED):
    """Trace-time unrolled training graph: returns the eDSL computation."""
    alice, bob, carole = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
    rep = pm.replicated_placement(name="rep", players=[alice, bob, carole])
    mir = pm.mirrored_placement(name="mirr", players=[alice, bob, carole])

    @pm.computation
    def train(x: pm.Argument(alice, dtype=pm.float64),
              y: pm.Argument(alice, dtype=pm.float64),
              w_0: pm.Argument(bob, dtype=pm.float64),
              b_0: pm.Argument(bob, dtype=pm.float64)):
        with alice:
            xf = pm.cast(x, dtype=fixed)
            yf = pm.cast(y, dtype=fixed)
            rows = [slice(i * batch_size, (i + 1) * batch_size) for i in range(n_batches)]
            xs = [xf[r, :] for r in rows]
            ys = [yf[r, :] for r in rows]
        with bob:
            w = pm.cast(w_0, dtype=fixed)
            b = pm.cast(b_0, dtype=fixed)
            eta = pm.cast(pm.constant(lr, dtype=pm.float64), dtype=fixed)
            mu = pm.cast(pm.constant(momentum, dtype=pm.float64), dtype=fixed)
        with mir:
            inv_n = pm.constant(1.0 / batch_size, dtype=fixed)
        with rep:
            xs = [pm.identity(xb) for xb in xs]  # share each batch exactly once
            velocity = None
            for xb, yb in zip(xs, ys):
                y_hat = pm.sigmoid(pm.dot(xb, w) + b)
                err = y_hat - yb
                g_w = pm.mul(pm.dot(pm.transpose(xb), err), inv_n)
                g_b = pm.mul(pm.sum(err, axis=0), inv_n)
                step_w, step_b = g_w * eta, g_b * eta
                if velocity is not None:
                    step_w = step_w + velocity[0] * mu
                    step_b = step_b + velocity[1] * mu
                velocity = (step_w, step_b)
                w = w - step_w
                b = b - step_b
        with bob:
            w_out = pm.cast(w, dtype=pm.float64)
            b_out = pm.cast(b, dtype=pm.float64)
        return w_out, b_out

    return train


def plaintext_training(x, y, batch_size, n_batches, lr=LEARNING_RATE, momentum=MOMENTUM):
    w = np.zeros((x.shape[1], 1))
    b = np.zeros((1, 1))
    vel = None
    for i in range(n_batches):
        xb, yb = x[i * batch_size:(i + 1) * batch_size], y[i * batch_size:(i + 1) * batch_size]
        y_hat = 1.0 / (1.0 + np.exp(-(xb @ w + b)))
        err = y_hat - yb
        gw, gb = xb.T @ err / batch_size, err.sum(0) / batch_size
        sw, sb = gw * lr, gb * lr
        if vel is not None:
            sw, sb = sw + vel[0] * momentum, sb + vel[1] * momentum
        vel = (sw, sb)
        w, b = w - sw, b - sb
    return w, b


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--n_iter", type=int, default=10)
    ap.add_argument("--n_exp", type=int, default=3)
    ap.add_argument("--runtime", choices=["local", "parties", "distributed"], default="local")
    ap.add_argument("--device", default=None)
    ap.add_argument("--devices", default=None,
                    help="parties runtime: comma-separated device per party")
    ap.add_argument("--graphs", action="store_true",
                    help="replay each evaluation as a captured hipGraph (runtime/graphs.py)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--json", default=None, help="append one JSON result line to this file")
    args = ap.parse_args(argv)

    rng = np.random.default_rng(args.seed)
    n_rows = args.batch_size * args.n_iter
    x = rng.standard_normal((n_rows, N_FEATURES))
    y = rng.integers(2, size=(n_rows, 1)).astype(np.float64)
    w0 = np.zeros((N_FEATURES, 1))
    b0 = np.zeros((1, 1))

    t_trace = time.perf_counter()
    comp = build_training(args.batch_size, args.n_iter)
    from moose_amd.runtime.local import to_native

    native = to_native(comp)
    t_trace = time.perf_counter() - t_trace
    ids = ["alice", "bob", "carole"]
    if args.runtime == "local":
        runtime = pm.LocalMooseRuntime(ids, device=args.device, use_graphs=args.graphs)
    elif args.runtime == "parties":
        import torch

        dev = args.device or ("cuda:0" if torch.cuda.is_available() else "cpu")
        devs = args.devices.split(",") if args.devices else [dev] * 3
        runtime = pm.LocalMooseRuntime(ids, device_map=dict(zip(ids, devs)),
                                       use_graphs=args.graphs, timeout=1200)
    else:
        runtime = pm.DistributedMooseRuntime(ids, timeout=1200)
    arguments = {"x": x, "y": y, "w_0": w0, "b_0": b0}

    runtime.evaluate_computation(native, arguments)  # warm-up (kernels, allocator)
    if args.runtime == "parties" and args.graphs:
        # the parties' tapes are recorded the second time a computation is seen (then
        # replayed): that evaluation is warm-up too
        runtime.evaluate_computation(native, arguments)
    session_s, wall_s = [], []
    outs = None
    for _ in range(args.n_exp):
        t0 = time.perf_counter()
        outs = runtime.evaluate_computation(native, arguments)
        wall_s.append(time.perf_counter() - t0)
        if args.runtime == "parties":  # the parties' threads run inside this call
            session_s.append(wall_s[-1])
        else:
            session_s.append(max(runtime.last_timings.values()) / 1e6)
    w_ref, b_ref = plaintext_training(x, y, args.batch_size, args.n_iter)
    vals = sorted(outs.values(), key=lambda v: -np.asarray(v).size)
    err = max(float(np.abs(np.asarray(vals[0]).reshape(w_ref.shape) - w_ref).max()),
              float(np.abs(np.asarray(vals[1]).reshape(b_ref.shape) - b_ref).max()))
    ref = REFERENCE_S.get((args.batch_size, args.n_iter))
    res = {
        "bench": "logreg_train", "batch_size": args.batch_size, "n_iter": args.n_iter,
        "n_features": N_FEATURES, "dtype": "fixed(24,40)/ring128", "runtime": args.runtime + ("+graphs" if args.graphs else ""),
        "device": (",".join(devs) if args.runtime == "parties"
                   else str(getattr(runtime, "device", runtime.__class__.__name__))),
        "session_s": {"min": min(session_s), "max": max(session_s),
                      "mean": statistics.mean(session_s)},
        "wall_s_mean": statistics.mean(wall_s), "trace_s": t_trace,
        "max_abs_err_vs_fp64": err, "reference_s": ref,
        "speedup_vs_reference": (ref / statistics.mean(session_s)) if ref else None,
    }
    print("MIN/MAX/VARIANCE/MEAN")
    var = statistics.variance(session_s) if len(session_s) > 1 else 0.0
    print(f"{min(session_s):.3f}/{max(session_s):.3f}/{var:.3f}/{statistics.mean(session_s):.3f}")
    print(json.dumps(res))
    if args.json:
        with open(args.json, "a") as f:
            f.write(json.dumps(res) + "\n")
    return res


if __name__ == "__main__":
    main()
