"""LR inference (tutorial model) with the three parties as threads of one process on one
GPU (``LocalMooseRuntime(device_map=...)``): p50 over ``--runs`` replays after 3 warm-ups.
Run it twice under ``rocprofv3 --kernel-trace --stats`` (``--runs 0`` and ``--runs N``) and
subtract to get the kernels of one replayed evaluation."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.getcwd())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--mode", default="parties", choices=["parties", "stacked"])
    a = ap.parse_args()
    import numpy as np
    import torch

    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.runtime.local import LocalMooseRuntime

    ids = ["alice", "bob", "carole"]
    tm = logistic_regression_tutorial(128)
    kw = {"device_map": {i: "cuda:0" for i in ids}, "timeout": 30} if a.mode == "parties" else {}
    rt = LocalMooseRuntime(ids, device="cuda:0", fixedpoint_ring=128, **kw)
    args = {"x": tm.x_test}
    for _ in range(3):
        r = rt.evaluate_computation(tm.computation, args)
    torch.cuda.synchronize()
    lat = []
    for _ in range(a.runs):
        t0 = time.perf_counter()
        r = rt.evaluate_computation(tm.computation, args)
        lat.append((time.perf_counter() - t0) * 1e3)
    lat.sort()
    err = float(np.abs(np.asarray(list(r.values())[0]) - tm.proba).max())
    rec = {"mode": a.mode, "runs": a.runs, "err": err,
           "p50_ms": lat[len(lat) // 2] if lat else None, "rounds": getattr(rt.last_stats, "rounds", None)}
    tapes = [t for _, t in getattr(rt, "_party_tapes", {}).values() if t]
    if tapes:
        t = tapes[0]
        rec["segments"] = t.segments
        rec["composed"] = t._composed is not None
        rec["actions"] = {k: sum(1 for x in t.actions if x[0] == k) for k in ("g", "rec", "cp")}
        iss = sorted(t.issue_s)
        rec["host_issue_ms_p50"] = iss[len(iss) // 2] * 1e3 if iss else None
        parts = getattr(t, "issue_parts", [])
        if parts:
            rec["issue_parts_ms_p50"] = [sorted(x)[len(x) // 2] * 1e3 for x in zip(*parts)]
        rec["graph_nodes"] = getattr(t, "graph_nodes", None)
        import time as _t
        # the device time of one replay alone (launch -> synchronize), no decode
        if t._composed is not None:
            ts = []
            for _ in range(10):
                torch.cuda.synchronize()
                t0 = _t.perf_counter()
                from moose_amd.ops import native as nat
                s = t.streams[0]
                for ex in t._composed:
                    nat.lib().mx_graph_launch(ex, s.cuda_stream)
                s.synchronize()
                ts.append((_t.perf_counter() - t0) * 1e3)
            rec["graph_only_ms_p50"] = sorted(ts)[5]
        rec["streams_mode"] = t._party_graphs is not None
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
