"""Independent-op batching in the interpreter (runtime/interpreter.Interpreter._batch_dots):
independent same-shape secret Dots run as ONE batched protocol instance
(fixedpoint.dot_many), with the same results as one instance per Dot."""
import numpy as np
import pytest

import moose_amd as pm
from moose_amd.protocols import fixedpoint as fxp
from moose_amd.runtime import interpreter as interp_mod


def _comp(k):
    alice, bob, carole = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(14, 23)

    @pm.computation
    def f(x: pm.Argument(alice, vtype=pm.TensorType(pm.float64)),
          y: pm.Argument(bob, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fx)
        with bob:
            yf = pm.cast(y, dtype=fx)
        with rep:
            zs = [pm.dot(xf, yf) for _ in range(k)]
            chain = pm.dot(zs[0], yf)  # depends on a batched result: not in the batch
            z = pm.add_n(zs + [chain])
        with carole:
            return pm.cast(z, dtype=pm.float64)

    return f


def test_independent_dots_batched(monkeypatch):
    calls = []
    orig = fxp.dot_many

    def spy(sess, pairs, f=None):
        calls.append(len(pairs))
        return orig(sess, pairs, f)

    monkeypatch.setattr(interp_mod.fxp, "dot_many", spy)
    rng = np.random.default_rng(0)
    x, y = rng.uniform(-1, 1, (6, 5)), rng.uniform(-1, 1, (5, 5))
    rt = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cpu")
    out = np.asarray(next(iter(rt.evaluate_computation(_comp(4), {"x": x, "y": y}).values())))
    assert calls == [4]
    np.testing.assert_allclose(out, 4 * (x @ y) + (x @ y) @ y, atol=1e-4)
    monkeypatch.setenv("MOOSEX_BATCH_DOTS", "0")
    calls.clear()
    out2 = np.asarray(next(iter(rt.evaluate_computation(_comp(4), {"x": x, "y": y}).values())))
    assert calls == []
    np.testing.assert_allclose(out, out2, atol=1e-4)


def _distinct_dots(k):
    alice, bob, carole = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(14, 23)

    @pm.computation
    def f(x: pm.Argument(alice, vtype=pm.TensorType(pm.float64)),
          y: pm.Argument(bob, vtype=pm.TensorType(pm.float64))):
        with alice:
            xs = [pm.cast(pm.mul(x, pm.constant(np.array([float(i + 1)]))), dtype=fx)
                  for i in range(k)]
        with bob:
            yf = pm.cast(y, dtype=fx)
        with rep:
            z = pm.add_n([pm.dot(xi, yf) for xi in xs])
        with carole:
            return pm.cast(z, dtype=pm.float64)

    return f


def test_independent_dots_batched_on_per_party_sessions(monkeypatch):
    """Parties as threads (one per-party SPMD session each): k independent Dots of distinct
    operands (6x5 . 5x3) run as ONE batched product and ONE dot tail -- the rounds of one
    product instead of k (BASELINE's "parallel" dot benchmark) -- with the plaintext
    values; MOOSEX_BATCH_DOTS=0 (and no lockstep) gives k times the rounds."""
    import os

    from moose_amd.runtime import interpreter as I
    from moose_amd.runtime.local import LocalMooseRuntime

    monkeypatch.setattr(I, "LOCKSTEP", False)

    ids = ["alice", "bob", "carole"]
    rng = np.random.default_rng(1)
    x, y = rng.uniform(-2, 2, (6, 5)), rng.uniform(-2, 2, (5, 3))
    want = sum((i + 1) * x for i in range(4)) @ y
    rounds = {}
    for flag in ("1", "0"):
        os.environ["MOOSEX_BATCH_DOTS"] = flag
        try:
            rt = LocalMooseRuntime(ids, device_map={i: "cpu" for i in ids}, seed=2)
            got = np.asarray(list(rt.evaluate_computation(_distinct_dots(4),
                                                          {"x": x, "y": y}).values())[0])
        finally:
            os.environ.pop("MOOSEX_BATCH_DOTS", None)
        np.testing.assert_allclose(got, want, atol=1e-4)
        rounds[flag] = rt.last_stats.rounds
    assert rounds["0"] >= rounds["1"] + 6, rounds  # 4 tails of 2 rounds -> one


def _scalar_factors():
    alice, bob, carole = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(24, 40)

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64)),
          c: pm.Argument(placement=bob, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fx)
        with bob:
            cf = pm.cast(c, dtype=fx)
        with rep:
            a = pm.mul(xf, cf)
            b = pm.add(pm.sub(a, cf), cf)
            z = pm.mul(cf, b)
        with carole:
            return pm.cast(z, dtype=pm.float64)

    return f


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_one_element_factors_broadcast_in_kernel(device, monkeypatch):
    """A one-element secret factor (a learning rate) times / plus a (5, 3) secret on the
    per-party sessions: broadcast inside the kernels (a stride-0 row of the batched tail,
    ring.binary2) instead of materialised -- bitwise the same outputs, and the values."""
    from moose_amd.runtime import interpreter as I
    from moose_amd.runtime.local import LocalMooseRuntime

    ids = ["alice", "bob", "carole"]
    rng = np.random.default_rng(4)
    args = {"x": rng.uniform(-3, 3, (5, 3)), "c": np.array(0.37)}
    outs = {}
    for flag in (False, True):
        monkeypatch.setattr(I, "BCAST_IN_KERNEL", flag)
        rt = LocalMooseRuntime(ids, device_map={i: device for i in ids}, seed=5,
                               use_graphs=False)
        outs[flag] = np.asarray(list(rt.evaluate_computation(_scalar_factors(), args).values())[0])
    assert np.array_equal(outs[True], outs[False])
    np.testing.assert_allclose(outs[True], 0.37 * 0.37 * args["x"], atol=1e-6)
