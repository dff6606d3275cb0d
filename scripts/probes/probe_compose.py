import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from moose_amd.runtime.local import LocalMooseRuntime
from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
IDS = ["alice", "bob", "carole"]
tm = logistic_regression_tutorial(128)
mode = sys.argv[1]
os.environ["MOOSEX_GRAPHS_DEBUG"] = "1"
rt = LocalMooseRuntime(IDS, device_map={i: "cuda:0" for i in IDS}, use_graphs=True)
for k in range(6):
    t0 = time.perf_counter()
    got = list(rt.evaluate_computation(tm.computation, {"x": tm.x_test}).values())[0]
    dt = (time.perf_counter() - t0) * 1e3
    tapes = [t for _, t in rt._party_tapes.values() if t]
    comp = tapes[0]._composed is not None if tapes else None
    print(mode, k, f"{dt:.2f} ms", "err", float(np.abs(got - tm.proba).max()), "composed", comp, flush=True)
