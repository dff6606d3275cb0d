"""Whole-evaluation hipGraph replay (runtime/graphs.py): replays with new inputs give the
same results as eager evaluation, use fresh keys, and really run from the graph."""
import importlib.util
import os
import warnings

import numpy as np
import pytest
import torch

import moose_amd as pm
from moose_amd.runtime import graphs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "benchmarks",
                                                                     f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_signature_distinguishes_shapes_and_values():
    a = graphs.signature({"x": np.zeros((2, 3)), "k": "key"})
    b = graphs.signature({"x": np.zeros((3, 3)), "k": "key"})
    c = graphs.signature({"x": np.ones((2, 3)), "k": "key"})
    assert a != b and a == c


def test_stager_rejects_data_dependent_uploads():
    rec = graphs._Recorder()
    rec(torch.arange(4), "cpu")
    rec(torch.arange(3), "cpu")
    st = graphs._Stager(rec.items, "cpu")
    assert torch.equal(st(torch.arange(3), "cpu"), torch.arange(3))  # skips a cached one
    with pytest.raises(graphs.CaptureError):
        st(torch.arange(4), "cpu")  # already behind it
    st = graphs._Stager(rec.items, "cpu")
    with pytest.raises(graphs.CaptureError):
        st(torch.arange(4) + 1, "cpu")


@pytest.mark.parametrize("t_graph,t_eager,want", [(1.0, 2.0, "graph"), (3.0, 2.0, "eager")])
def test_adaptive_replay_keeps_the_faster_mode(monkeypatch, t_graph, t_eager, want):
    """Adaptive mode (MOOSEX_GRAPHS_PROBES=k): after the capture a plan times k replays and
    k eager evaluations, then keeps the faster mode."""
    monkeypatch.setattr(graphs, "PROBES", 3)
    plan = graphs.GraphPlan.__new__(graphs.GraphPlan)
    plan.t_graph, plan.t_eager, plan.decision, plan._warm = [], [], None, False
    seen = []
    for _ in range(2 * graphs.PROBES + 1):
        mode = plan.next_mode()
        seen.append(mode)
        if mode != "graph":  # the first replay is untimed
            (plan.t_graph if mode == "probe" else plan.t_eager).append(
                t_graph if mode == "probe" else t_eager)
    assert seen == ["graph"] + ["probe", "eager"] * graphs.PROBES
    assert plan.next_mode() == want and plan.decision == want


@pytest.mark.gpu
def test_logreg_training_replays_from_graph():
    L = _load("logreg_train")
    bs, n_it, nf = 64, 3, 100
    from moose_amd.runtime.local import to_native

    native = to_native(L.build_training(bs, n_it, n_features=nf))
    rt = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", use_graphs=True)
    rng = np.random.default_rng(3)
    with warnings.catch_warnings():
        warnings.filterwarnings("error", message="hipGraph capture failed")
        for rep in range(3):
            x = rng.standard_normal((bs * n_it, nf))
            y = rng.integers(2, size=(bs * n_it, 1)).astype(np.float64)
            outs = rt.evaluate_computation(native, {"x": x, "y": y,
                                                    "w_0": np.zeros((nf, 1)),
                                                    "b_0": np.zeros((1, 1))})
            w_ref, b_ref = L.plaintext_training(x, y, bs, n_it)
            vals = sorted(outs.values(), key=lambda v: -np.asarray(v).size)
            np.testing.assert_allclose(vals[0].reshape(w_ref.shape), w_ref, atol=1e-5)
            np.testing.assert_allclose(vals[1].reshape(b_ref.shape), b_ref, atol=1e-5)
    plans = list(rt._graphs.plans.values())
    assert len(plans) == 1 and plans[0].replays == 2


@pytest.mark.gpu
def test_graph_replay_refreshes_keys():
    D = _load("dot_product")
    from moose_amd.runtime.local import to_native

    native = to_native(D.build("seq", 2))
    rt = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", use_graphs=True)
    args = {"x_arg": np.ones((8, 8)), "y_arg": np.identity(8)}
    rt.evaluate_computation(native, args)
    plan = next(iter(rt._graphs.plans.values()))
    k0 = plan.keys.t.clone()
    out = rt.evaluate_computation(native, args)
    assert not torch.equal(k0, plan.keys.t)
    np.testing.assert_allclose(next(iter(out.values())), np.ones((8, 8)), atol=1e-6)


@pytest.mark.gpu
def test_default_runtime_replays_dispatch_bound_evaluations():
    """LocalMooseRuntime with no flags on a GPU (auto mode): the first evaluation runs
    eagerly, the second (same signature, dispatch-bound) is captured, later ones replay --
    with fresh inputs and correct results."""
    import time

    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial

    tm = logistic_regression_tutorial(128)
    rt = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda")
    assert rt.use_graphs == "auto"
    lat = []
    for i in range(12):
        t0 = time.perf_counter()
        out = rt.evaluate_computation(tm.computation, {"x": tm.x_test})
        lat.append((time.perf_counter() - t0) * 1e3)
        got = np.asarray(list(out.values())[0])
        assert np.abs(got - tm.proba).max() < 1e-3
        assert bool(rt._graphs.plans) == (i >= 1)
    plan = next(iter(rt._graphs.plans.values()))
    assert plan.replays == 10
    warm = sorted(lat[3:])
    print(f"default LocalMooseRuntime LR p50 {warm[len(warm) // 2]:.3f} ms")


@pytest.mark.gpu
def test_small_constants_uploaded_and_encoded_once():
    """A computation's small tensor constants (the tutorial model's weights and intercept)
    are uploaded and fixed-point encoded once per device and reused by later evaluations,
    eager and replayed; the predictions stay right."""
    import numpy as np

    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.ops import ring as R
    from moose_amd.runtime import interpreter as I
    from moose_amd.runtime.local import LocalMooseRuntime

    tm = logistic_regression_tutorial(128)
    for graphs in (False, True):
        rt = LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", use_graphs=graphs)
        outs = [list(rt.evaluate_computation(tm.computation, {"x": tm.x_test}).values())[0]
                for _ in range(4)]
        assert I._CONST_LV and R._ENCODED_CONSTS
        n = (len(I._CONST_LV), len(R._ENCODED_CONSTS))
        outs.append(list(rt.evaluate_computation(tm.computation, {"x": tm.x_test}).values())[0])
        assert (len(I._CONST_LV), len(R._ENCODED_CONSTS)) == n
        for o in outs:
            assert np.abs(np.asarray(o) - tm.proba).max() < 1e-4


@pytest.mark.gpu
def test_seeded_auto_replays_match_seeded_eager_bitwise():
    """a seeded runtime in the default auto mode replays from its third
    evaluation; every replay must equal a seeded eager evaluation bitwise (the replay
    re-draws the seeded keys exactly as a fresh seeded session's setup would)."""
    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial

    tm = logistic_regression_tutorial(128)
    args = {"x": tm.x_test}
    eager = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", seed=11,
                                 use_graphs=False)
    want = np.asarray(list(eager.evaluate_computation(tm.computation, args).values())[0])
    auto = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", seed=11)
    assert auto.use_graphs == "auto"
    for i in range(5):
        got = np.asarray(list(auto.evaluate_computation(tm.computation, args).values())[0])
        assert np.array_equal(got, want), (i, np.abs(got - want).max())
    plan = next(iter(auto._graphs.plans.values()))
    assert plan.replays >= 3
