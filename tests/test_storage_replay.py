"""Storage-backed computations replay (runtime/storage_tap.py; VERDICT r5 "missing" 2).

The reference runs Load / Save as dataflow tasks of the session like any other operation
(/root/reference/moose/src/execution/asynchronous.rs:149-238, 456-466); here a replayed
evaluation (stacked hipGraph plan, per-party tapes, multi-process SPMD plans) serves them
at its edges: loaded values are static buffers refreshed from storage before each replay,
saved values are read back after it.  A stored value of a new shape re-captures."""
import numpy as np
import pytest

import moose_amd as pm
from moose_amd.runtime import storage_tap as ST
from moose_amd.runtime.local import LocalMooseRuntime
from moose_amd.runtime.local import to_native

FIXED = pm.fixed(8, 27)
IDS = ["x-owner", "y-owner", "model-owner"]


def linreg_comp():
    """The reference's linear-regression example (pymoose/examples/linear-regression/
    linreg_test.py, mse metric): X and y loaded from the owners' storage by string-argument
    keys, host inverse, replicated fit and metrics, three results saved."""
    x_owner, y_owner, model_owner = (pm.host_placement(name=n) for n in IDS)
    rep = pm.replicated_placement(players=[x_owner, y_owner, model_owner], name="rep")

    @pm.computation
    def comp(x_uri: pm.Argument(placement=x_owner, vtype=pm.StringType()),
             y_uri: pm.Argument(placement=y_owner, vtype=pm.StringType()),
             w_uri: pm.Argument(placement=model_owner, vtype=pm.StringType()),
             metric_uri: pm.Argument(placement=model_owner, vtype=pm.StringType()),
             rsquared_uri: pm.Argument(placement=model_owner, vtype=pm.StringType())):
        with x_owner:
            X = pm.atleast_2d(pm.load(x_uri, dtype=pm.float64), to_column_vector=True)
            bias = pm.ones(pm.shape(X)[0:1], dtype=pm.float64)
            X_b = pm.concatenate([pm.expand_dims(bias, 1), X], axis=1)
            A = pm.inverse(pm.dot(pm.transpose(X_b), X_b))
            B = pm.dot(A, pm.transpose(X_b))
            X_b = pm.cast(X_b, dtype=FIXED)
            B = pm.cast(B, dtype=FIXED)
        with y_owner:
            y_true = pm.atleast_2d(pm.load(y_uri, dtype=pm.float64), to_column_vector=True)
            y_mean = pm.mean(y_true)
            totals_ss = pm.sum(pm.square(pm.sub(y_true, y_mean)), axis=0)
            y_true = pm.cast(y_true, dtype=FIXED)
        with rep:
            w = pm.dot(B, y_true)
            y_pred = pm.dot(X_b, w)
            mse = pm.mean(pm.square(pm.sub(y_pred, y_true)), axis=0)
            residuals_ss = pm.sum(pm.square(pm.sub(y_true, y_pred)), axis=0)
        with model_owner:
            residuals_ss = pm.cast(residuals_ss, dtype=pm.float64)
            rsq = pm.sub(pm.constant(1.0, dtype=pm.float64), pm.div(residuals_ss, totals_ss))
            w = pm.cast(w, dtype=pm.float64)
            mse = pm.cast(mse, dtype=pm.float64)
            res = (pm.save(w_uri, w), pm.save(metric_uri, mse), pm.save(rsquared_uri, rsq))
        return res

    return comp


ARGS = {"x_uri": "x_data", "y_uri": "y_data", "w_uri": "regression_weights",
        "metric_uri": "metric_result", "rsquared_uri": "rsquared_result"}
OUT_KEYS = ("regression_weights", "metric_result", "rsquared_result")


def _data(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, 1))
    return x, x[:, 0] * 3.0 + 10.0


def test_storage_ops_resolve_constant_and_argument_keys():
    comp = to_native(linreg_comp(), 128)
    loads, saves = ST.storage_ops(comp, ARGS)
    assert {(h, k) for _, h, k, _ in loads} == {("x-owner", "x_data"), ("y-owner", "y_data")}
    assert {(h, k) for _, h, k in saves} == {("model-owner", k) for k in OUT_KEYS}
    assert ST.capturable(comp, ARGS)
    storage = {"x-owner": {"x_data": np.zeros((5, 1))}, "y-owner": {"y_data": np.zeros(5)}}
    sig = ST.signature(comp, storage, arguments=ARGS)
    storage["x-owner"]["x_data"] = np.zeros((6, 1))
    assert ST.signature(comp, storage, arguments=ARGS) != sig  # a new shape: a new plan


def test_load_of_a_key_saved_by_the_same_evaluation_stays_eager():
    alice = pm.host_placement("alice")

    @pm.computation
    def f():
        with alice:
            v = pm.load("k", dtype=pm.float64)
            return pm.save("k", pm.add(v, v))

    assert not ST.capturable(to_native(f, 128), {})


def _run_linreg(rt, storage_of, n, seed):
    x, y = _data(n, seed)
    rt.write_value_to_storage("x-owner", "x_data", x)
    rt.write_value_to_storage("y-owner", "y_data", y)
    rt.evaluate_computation(linreg_comp_cached(), ARGS)
    return [np.asarray(rt.read_value_from_storage("model-owner", k)) for k in OUT_KEYS]


_COMP = []


def linreg_comp_cached():
    if not _COMP:
        _COMP.append(linreg_comp())
    return _COMP[0]


def _mk(kind, device, graphs):
    storage = {i: {} for i in IDS}
    if kind == "parties":
        return LocalMooseRuntime(IDS, storage_mapping=storage, seed=7, use_graphs=graphs,
                                 device_map={i: device for i in IDS})
    return LocalMooseRuntime(IDS, storage_mapping=storage, seed=7, use_graphs=graphs,
                             device=device)


@pytest.mark.parametrize("kind", ["stacked", "parties"])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_linreg_example_replays_bitwise_equal_eager(device, kind):
    """The reference's linreg example fed from storage: every evaluation's saved results
    equal the eager (seeded) ones bitwise -- from the second evaluation on a replay on a GPU
    -- also across a stored shape change (re-captured) and back."""
    eager = _mk(kind, device, False)
    rt = _mk(kind, device, True)
    for n, seed in ((10, 1), (10, 2), (10, 3), (12, 4), (12, 5), (12, 6), (10, 7)):
        want = _run_linreg(eager, None, n, seed)
        got = _run_linreg(rt, None, n, seed)
        for a, b in zip(got, want):
            assert a.shape == b.shape and np.array_equal(a, b), (n, seed, a, b)
        w = want[0].reshape(-1)
        assert abs(w[0] - 10.0) < 1e-3 and abs(w[1] - 3.0) < 1e-3
    if device != "cpu":
        if kind == "stacked":
            plans = rt._graphs.plans
            assert len(plans) == 2 and all(p.replays >= 1 for p in plans.values())
        else:
            tapes = [t for _, t in rt._party_tapes.values() if t is not False]
            assert len(tapes) == 2 and all(t.tapes[0].replays >= 1 for t in tapes)


def _lr_storage_comp(coef, intercept):
    alice, bob, carole = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    mir = pm.mirrored_placement(name="mir", players=[alice, bob, carole])
    fx = pm.fixed(24, 40)

    @pm.computation
    def f():
        with alice:
            x = pm.cast(pm.load("x", dtype=pm.float64), dtype=fx)
        w = pm.cast(pm.constant(coef, dtype=pm.float64, placement=mir), dtype=fx, placement=mir)
        b = pm.cast(pm.constant(intercept, dtype=pm.float64, placement=mir), dtype=fx,
                    placement=mir)
        with rep:
            p = pm.sigmoid(pm.add(pm.dot(x, w), b))
        with bob:
            return pm.save("proba", pm.cast(p, dtype=pm.float64))

    return f


@pytest.mark.parametrize("kind", ["stacked", "parties"])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_storage_fed_lr_inference_replays(device, kind):
    """A private LR inference whose input comes from alice's storage and whose probabilities
    go to bob's: replayed evaluations equal the eager (seeded) ones bitwise and sklearn's
    within 1e-6."""
    rng = np.random.default_rng(3)
    coef = rng.normal(size=(10, 1))
    icpt = np.array([0.25])
    comp = _lr_storage_comp(coef, icpt)
    ids = ["alice", "bob", "carole"]

    def mk(graphs):
        st = {i: {} for i in ids}
        kw = {"device_map": {i: device for i in ids}} if kind == "parties" else {"device": device}
        return LocalMooseRuntime(ids, storage_mapping=st, seed=9, use_graphs=graphs, **kw)

    eager, rt = mk(False), mk(True)
    for k in range(4):
        x = rng.normal(size=(200, 10))
        for r in (eager, rt):
            r.write_value_to_storage("alice", "x", x)
            r.evaluate_computation(comp, {})
        a = np.asarray(rt.read_value_from_storage("bob", "proba"))
        b = np.asarray(eager.read_value_from_storage("bob", "proba"))
        assert np.array_equal(a, b), k
        want = 1.0 / (1.0 + np.exp(-(x @ coef + icpt)))
        assert np.abs(a - want).max() < 1e-6
    if device != "cpu":
        if kind == "stacked":
            assert any(p.replays >= 2 for p in rt._graphs.plans.values())
        else:
            (_, tapes), = rt._party_tapes.values()
            assert tapes is not False and tapes.tapes[0].replays >= 2


@pytest.mark.parametrize("kind", ["stacked", "parties"])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_storage_fed_tutorial_lr_equals_argument_fed(device, kind):
    """The tutorial's ONNX LR with x read from alice's storage (storage_tap.storage_fed):
    every evaluation (replayed from the second on a GPU) bitwise equal to the argument-fed
    one under the same seed."""
    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial

    tm = logistic_regression_tutorial(128)
    native = to_native(tm.computation, 128)
    x_arg = [op for op in native.operations if op.kind == "Input"]
    names = {op.attrs.get("arg_name") or op.name for op in x_arg}
    fed = ST.storage_fed(native, names)
    assert not any(op.kind == "Input" for op in fed.operations)
    ids = ["alice", "bob", "carole"]
    host = x_arg[0].placement.owner

    def mk():
        kw = {"device_map": {i: device for i in ids}} if kind == "parties" else {"device": device}
        return LocalMooseRuntime(ids, storage_mapping={i: {} for i in ids}, seed=4,
                                 use_graphs=True, **kw)

    a_rt, s_rt = mk(), mk()
    for _ in range(3):
        want = a_rt.evaluate_computation(native, {n: tm.x_test for n in names})
        for n in names:
            s_rt.write_value_to_storage(host, n, tm.x_test)
        got = s_rt.evaluate_computation(fed, {})
        assert set(got) == set(want)
        for k in want:
            assert np.array_equal(np.asarray(got[k]), np.asarray(want[k])), k
