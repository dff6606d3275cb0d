"""Launch only the composed party graph of a workload N times (after the warm-up that
records it), so a rocprofv3 kernel trace of --launches 0 and --launches N differs by
exactly N replays' kernels (scripts/probes/kernel_table.py makes the table).

    python scripts/probes/graph_kernels.py --workload logreg --launches 20
"""
import argparse
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "benchmarks"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["lr", "logreg"], default="logreg")
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--n_iter", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch

    from moose_amd.ops import native as nat
    from moose_amd.runtime.local import LocalMooseRuntime, to_native

    ids = ["alice", "bob", "carole"]
    rt = LocalMooseRuntime(ids, device_map={i: "cuda:0" for i in ids}, use_graphs=True,
                           timeout=120)
    if a.workload == "lr":
        from moose_amd.models.predictors.tutorial import logistic_regression_tutorial

        tm = logistic_regression_tutorial(128)
        comp, args = tm.computation, {"x": tm.x_test}
    else:
        from logreg_train import N_FEATURES, build_training

        rng = np.random.default_rng(0)
        n = 128 * a.n_iter
        comp = to_native(build_training(128, a.n_iter))
        args = {"x": rng.standard_normal((n, N_FEATURES)),
                "y": rng.integers(2, size=(n, 1)).astype(np.float64),
                "w_0": np.zeros((N_FEATURES, 1)), "b_0": np.zeros((1, 1))}
    for _ in range(3):
        rt.evaluate_computation(comp, args)
    torch.cuda.synchronize()
    (_, tapes), = rt._party_tapes.values()
    assert tapes is not False and tapes._composed is not None, "no composed graph"
    s = tapes.streams[0]
    for _ in range(a.launches):
        for ex in tapes._composed:
            nat.check(nat.lib().mx_graph_launch(ex, s.cuda_stream), "graph launch")
    s.synchronize()
    print({"workload": a.workload, "launches": a.launches, "graph_nodes": tapes.graph_nodes},
          flush=True)


if __name__ == "__main__":
    main()
