"""Latency of a computation with independent branches (B secret sigmoid(x.w_i) chains
summed at the end) with 1..L dataflow lanes (runtime/lanes.py), eager and with hipGraph
replay.  One JSON line per configuration."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--branches", type=int, default=8)
    ap.add_argument("--rows", type=int, default=200)
    ap.add_argument("--runs", type=int, default=30)
    ap.add_argument("--lanes", default="1,2,4")
    a = ap.parse_args()
    import moose_amd as pm
    from tests.test_lanes import _wide_comp

    f, x, ref = _wide_comp(a.branches, a.rows)
    for graphs in (False, True):
        for lanes in [int(v) for v in a.lanes.split(",")]:
            rt = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda",
                                      use_graphs=graphs, lanes=lanes)
            for _ in range(3):
                rt.evaluate_computation(f, {"x": x})
            lat = []
            for _ in range(a.runs):
                t0 = time.perf_counter()
                r = rt.evaluate_computation(f, {"x": x})
                lat.append(time.perf_counter() - t0)
            err = float(np.abs(np.asarray(list(r.values())[0]) - ref).max())
            print(json.dumps({"bench": "independent_branches", "branches": a.branches,
                              "rows": a.rows, "lanes": lanes, "graphs": graphs,
                              "p50_ms": float(np.median(lat)) * 1e3, "max_abs_err": err,
                              "captured": bool(graphs and rt._graphs.plans)}),
                  flush=True)


if __name__ == "__main__":
    main()
