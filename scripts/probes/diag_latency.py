"""Diagnostics for the latency path (GPU): (1) where the hipGraph replay time of a
1000^2 replicated dot goes (argument upload, key refresh, replay, output decode);
(2) which Python call sites launch ATen kernels / memcpys during one private LR
inference (torch profiler with stacks)."""
import collections
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def graph_breakdown(n=1000):
    import moose_amd as pm
    from moose_amd.runtime.local import to_native

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))
    import dot_product as dp

    native = to_native(dp.build("seq", 1))
    args = {"x_arg": np.ones((n, n)), "y_arg": np.identity(n)}
    rt = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", use_graphs=True)
    rt.evaluate_computation(native, args)
    rt.evaluate_computation(native, args)
    plan = next(iter(rt._graphs.plans.values()))
    for _ in range(3):
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        for k, v in args.items():
            st = plan.static[k]
            st.copy_(torch.from_numpy(np.asarray(v)))
        torch.cuda.synchronize(); t.append(time.perf_counter())
        plan.keys.refresh()
        torch.cuda.synchronize(); t.append(time.perf_counter())
        for g in plan.graphs:
            g.replay()
        torch.cuda.synchronize(); t.append(time.perf_counter())
        plan._decode(plan.interp, plan.outs)
        torch.cuda.synchronize(); t.append(time.perf_counter())
        d = np.diff(t) * 1e3
        print(f"graph replay n={n}: upload {d[0]:.2f} ms, key refresh {d[1]:.2f}, "
              f"replay {d[2]:.2f} ({len(plan.graphs)} graphs), decode {d[3]:.2f}", flush=True)
    for _ in range(3):
        t0 = time.perf_counter()
        rt.evaluate_computation(native, args)
        print(f"evaluate (graphs) {1e3 * (time.perf_counter() - t0):.2f} ms, "
              f"last_timings {rt.last_timings['alice'] / 1e3:.2f} ms", flush=True)
    rt2 = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", use_graphs=False)
    rt2.evaluate_computation(native, args)
    for _ in range(3):
        t0 = time.perf_counter()
        rt2.evaluate_computation(native, args)
        print(f"evaluate (eager) {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)


def lr_sources():
    from sklearn.datasets import make_classification
    from sklearn.linear_model import LogisticRegression
    from sklearn.model_selection import train_test_split
    from torch.profiler import ProfilerActivity
    from torch.profiler import profile

    from moose_amd.models import predictors
    from moose_amd.runtime.local import LocalMooseRuntime

    X, y = make_classification(n_samples=1000, n_features=10, n_classes=2, random_state=5)
    X_train, X_test, y_train, _ = train_test_split(X, y, test_size=0.2, random_state=5)
    lg = LogisticRegression().fit(X_train, y_train)
    model = predictors.LinearClassifier(np.stack([-lg.coef_[0], lg.coef_[0]]),
                                        np.array([-lg.intercept_[0], lg.intercept_[0]]),
                                        predictors.PostTransform.SIGMOID)
    comp = model.predictor_factory(predictors.DEFAULT_FIXED_DTYPE)
    rt = LocalMooseRuntime(["alice", "bob", "carole"], device="cuda")
    for _ in range(3):
        rt.evaluate_computation(comp, {"x": X_test})
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as p:
        rt.evaluate_computation(comp, {"x": X_test})
    torch.cuda.synchronize()
    where = collections.Counter()
    for e in p.events():
        if e.device_type.name != "CPU" or not e.name.startswith("aten::"):
            continue
        if e.name not in ("aten::copy_", "aten::cat", "aten::stack", "aten::contiguous",
                          "aten::clone", "aten::to", "aten::_to_copy", "aten::zeros",
                          "aten::bitwise_and", "aten::__lshift__", "aten::bitwise_left_shift",
                          "aten::__rshift__", "aten::bitwise_xor", "aten::fill_",
                          "aten::index", "aten::where", "aten::add", "aten::mul", "aten::sub"):
            continue
        frames = [f for f in (e.stack or []) if "moose_amd" in f]
        where[(e.name, frames[0].split("moose_amd/")[-1] if frames else "?")] += 1
    for k, v in where.most_common(40):
        print(v, k)
    kern = collections.Counter(e.name[:60] for e in p.events() if e.device_type.name == "CUDA")
    print("device events per inference:", sum(kern.values()))
    for k, v in kern.most_common(25):
        print("  ", v, k)


if __name__ == "__main__":
    graph_breakdown()
    lr_sources()
