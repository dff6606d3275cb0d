"""Replicated dot-product benchmarks: k sequential or k parallel secret matmuls.

Workload parity with the reference's ``benchmarks/pymoose/dot_product.py``: ``x`` (ones)
on alice and ``y`` (identity) on bob, both cast to ``fixed(8, 27)``, shared into the
replicated placement; "seq" chains ``z_i = z_{i-1} . y``, "parallel" sums k independent
``x . y``; the result is revealed to carole.  BASELINE.md tabulates the reference's
seconds per evaluation (3 gRPC workers, max over workers) for n in {1, 10, 100, 1000} and
k in {1, 10, 100}; ``--sweep`` reproduces that whole table for our runtime.

Usage::

    python benchmarks/dot_product.py --c seq --s 100 --c_arg 10 --n 3
    python benchmarks/dot_product.py --sweep [--max_n 1000] [--json out.jsonl]
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

FIXED = pm.fixed(8, 27)

# reference seconds from BASELINE.md keyed (mode, k, n)
REFERENCE_S = {
    ("seq", 1, 1): 0.0039, ("seq", 1, 10): 0.0027, ("seq", 1, 100): 0.102,
    ("seq", 1, 1000): 5.910, ("seq", 10, 1): 0.017, ("seq", 10, 10): 0.0180,
    ("seq", 10, 100): 0.717, ("seq", 10, 1000): 54.588, ("seq", 100, 1): 0.099,
    ("seq", 100, 10): 0.1232, ("seq", 100, 100): 0.675, ("seq", 100, 1000): 545.675,
    ("parallel", 1, 1): 0.039, ("parallel", 1, 10): 0.004, ("parallel", 1, 100): 0.006,
    ("parallel", 1, 1000): 5.844, ("parallel", 10, 1): 0.010, ("parallel", 10, 10): 0.0107,
    ("parallel", 10, 100): 0.016, ("parallel", 10, 1000): 11.110,
    ("parallel", 100, 1): 0.041, ("parallel", 100, 10): 0.066,
    ("parallel", 100, 100): 0.135, ("parallel", 100, 1000): 163.098,
}


def build(mode: str, k: int):
    alice, bob, carole = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
    rep = pm.replicated_placement(name="rep", players=[alice, bob, carole])

    @pm.computation
    def comp(x_arg: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64)),
             y_arg: pm.Argument(placement=bob, vtype=pm.TensorType(pm.float64))):
        with alice:
            x = pm.cast(x_arg, dtype=FIXED)
        with bob:
            y = pm.cast(y_arg, dtype=FIXED)
        with rep:
            y_rep = pm.identity(y)
            if mode == "seq":
                z = pm.dot(x, y_rep)
                for _ in range(k - 1):
                    z = pm.dot(z, y_rep)
            else:
                x_rep = pm.identity(x)
                z = pm.add_n([pm.dot(x_rep, y_rep) for _ in range(k)])
        with carole:
            return pm.cast(z, pm.float64)

    return comp


def run_one(runtime, mode, n, k, n_iter, parties=False):
    from moose_amd.runtime.local import to_native

    native = to_native(build(mode, k))
    x = np.ones((n, n))
    y = np.identity(n)
    args = {"x_arg": x, "y_arg": y}
    runtime.evaluate_computation(native, args)  # warm-up
    if parties:
        # the parties' tapes are recorded the second time a computation is seen
        runtime.evaluate_computation(native, args)
    elif getattr(runtime, "use_graphs", False):
        # hipGraph plans: capture, then the adaptive probes (runtime/graphs.py) decide
        # between replay and eager before the timed evaluations
        from moose_amd.runtime.graphs import PROBES

        for _ in range(2 * PROBES + 2):
            runtime.evaluate_computation(native, args)
    times = []
    out = None
    for _ in range(n_iter):
        t0 = time.perf_counter()
        out = runtime.evaluate_computation(native, args)
        if parties:  # the parties' threads (or replay) run inside this call
            times.append(time.perf_counter() - t0)
        else:
            times.append(max(runtime.last_timings.values()) / 1e6)
    z = np.asarray(next(iter(out.values())))
    expect = x * (k if mode == "parallel" else 1)
    ref = REFERENCE_S.get((mode, k, n))
    mean = statistics.mean(times)
    return {"bench": "dot_product", "mode": mode, "n": n, "k": k, "seconds_mean": mean,
            "seconds_min": min(times), "seconds_median": statistics.median(times),
            "seconds_all": times, "max_abs_err": float(np.abs(z - expect).max()),
            "reference_s": ref, "speedup_vs_reference": (ref / mean) if ref else None}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--c", dest="mode", choices=["seq", "parallel"], default="parallel")
    ap.add_argument("--s", dest="n", type=int, default=1)
    ap.add_argument("--c_arg", dest="k", type=int, default=1)
    ap.add_argument("--n", dest="n_iter", type=int, default=3)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--max_n", type=int, default=1000)
    ap.add_argument("--runtime", choices=["local", "parties", "distributed"], default="local",
                    help="parties: each party a thread on its own HIP stream running the "
                         "per-party protocol (--devices: one device per party)")
    ap.add_argument("--device", default=None)
    ap.add_argument("--devices", default=None)
    ap.add_argument("--graphs", action="store_true",
                    help="replay each evaluation as a captured hipGraph (runtime/graphs.py)")
    ap.add_argument("--json", default=None)
    args = ap.parse_args(argv)

    ids = ["alice", "bob", "carole"]
    devs = None
    if args.runtime == "local":
        runtime = pm.LocalMooseRuntime(ids, device=args.device, use_graphs=args.graphs)
    elif args.runtime == "parties":
        import torch

        dev = args.device or ("cuda:0" if torch.cuda.is_available() else "cpu")
        devs = args.devices.split(",") if args.devices else [dev] * 3
        runtime = pm.LocalMooseRuntime(ids, device_map=dict(zip(ids, devs)),
                                       use_graphs=args.graphs, timeout=1200)
    else:
        runtime = pm.DistributedMooseRuntime(ids, timeout=1800)
    if args.sweep:
        cases = [(m, k, n) for m in ("seq", "parallel") for k in (1, 10, 100)
                 for n in (1, 10, 100, 1000) if n <= args.max_n]
    else:
        cases = [(args.mode, args.k, args.n)]
    results = []
    for mode, k, n in cases:
        res = run_one(runtime, mode, n, k, args.n_iter, parties=args.runtime == "parties")
        res["runtime"] = args.runtime + ("+graphs" if args.graphs else "")
        res["device"] = (",".join(devs) if devs else str(getattr(runtime, "device",
                                                                 "distributed")))
        results.append(res)
        print(json.dumps(res), flush=True)
        if args.json:
            with open(args.json, "a") as f:
                f.write(json.dumps(res) + "\n")
    return results


if __name__ == "__main__":
    main()
