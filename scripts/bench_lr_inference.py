"""Private logistic-regression inference latency (BASELINE config 4, the reference's
``tutorials/ml-inference-with-onnx`` setup): sklearn LogisticRegression on
make_classification(1000 samples, 10 features, 2 classes, random_state=5), 80/20 split;
the 200 test rows are secret-shared from alice, scored on the replicated placement
(public weights, secure sigmoid) and the probabilities opened to bob.

Prints one JSON line with p50/p90 latency of the whole computation (share -> predict ->
reveal) over ``--runs`` evaluations, and the max deviation from sklearn's
``predict_proba``.  Single process: the three parties are stacked on one device.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--device", default=None)
    ap.add_argument("--ring", type=int, default=128, choices=(64, 128))
    ap.add_argument("--graphs", action="store_true", help="replay captured hipGraphs")
    ap.add_argument("--cprofile", default=None, help="write a host-side cProfile summary")
    ap.add_argument("--parties", action="store_true",
                    help="the three parties as threads of this process, one stream each "
                         "(LocalMooseRuntime device_map; replayed per-party tapes)")
    a = ap.parse_args()
    import torch
    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.runtime.local import LocalMooseRuntime

    # the tutorial's path: sklearn model -> ONNX -> predictors.from_onnx (tutorial.py)
    tm = logistic_regression_tutorial(a.ring)
    dtype, comp, X_test = tm.dtype, tm.computation, tm.x_test
    dev = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    extra = {}
    if a.parties:
        extra = {"device_map": {r: "cuda:0" if dev == "cuda" else dev
                                for r in ("alice", "bob", "carole")}, "timeout": 30}
    rt = LocalMooseRuntime(["alice", "bob", "carole"], device=dev, fixedpoint_ring=a.ring,
                           use_graphs=a.graphs, **extra)
    args = {"x": X_test}
    for _ in range(a.warmup):
        out = rt.evaluate_computation(comp, args)
    lat = []
    prof = None
    if a.cprofile:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    for _ in range(a.runs):
        t0 = time.perf_counter()
        out = rt.evaluate_computation(comp, args)
        lat.append(time.perf_counter() - t0)
    if prof is not None:
        import io
        import pstats

        prof.disable()
        buf = io.StringIO()
        st = pstats.Stats(prof, stream=buf)
        st.sort_stats("tottime").print_stats(45)
        st.sort_stats("cumulative").print_stats(60)
        with open(a.cprofile, "w") as f:
            f.write(buf.getvalue())
    pred = np.asarray(list(out.values())[0])
    err = float(np.abs(pred - tm.proba).max())
    lat = np.sort(np.asarray(lat)) * 1e3
    print(json.dumps({
        "metric": "private LR inference p50 latency", "value": float(np.median(lat)),
        "unit": "ms", "p90_ms": float(lat[int(0.9 * (len(lat) - 1))]), "runs": a.runs,
        "higher_is_better": False, "batch": int(X_test.shape[0]), "features": 10,
        "device": dev, "ring": a.ring, "graphs": a.graphs,
        "fixed": [dtype.integral_precision, dtype.fractional_precision], "max_abs_err_vs_sklearn": err,
        "data": "make_classification(random_state=5), sklearn LogisticRegression -> ONNX "
                "-> predictors.from_onnx",
        "layout": ("three party threads, one stream each, on one GPU" if a.parties
                   else "stacked 3-party session on one GPU"),
    }))


if __name__ == "__main__":
    main()
