"""Independent-op batching in the interpreter (runtime/interpreter.Interpreter._batch_dots):
independent same-shape secret Dots run as ONE batched protocol instance
(fixedpoint.dot_many), with the same results as one instance per Dot."""
import numpy as np

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
