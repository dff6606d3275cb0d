"""The in-place row stacks of the stacked session (poly_eval powers, exp2 product tree;
the mul kernel reads row slices / broadcast rows as views) compute bitwise the same shares
as the generic slice/concat path: with equal seeds the revealed results are identical."""
import numpy as np
import pytest

import moose_amd as pm
from moose_amd.protocols import fixedpoint as fxp

pytestmark = pytest.mark.gpu


def _comp(fn):
    alice, bob, carole = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=pm.fixed(24, 40))
        with rep:
            y = fn(xf)
        with carole:
            out = pm.cast(y, dtype=pm.float64)
        return out

    return f


@pytest.mark.parametrize("name,fn,ref", [("sigmoid", pm.sigmoid, lambda x: 1 / (1 + np.exp(-x))),
                                         ("exp", pm.exp, np.exp)])
def test_rows_path_bitwise_equal(monkeypatch, name, fn, ref):
    x = np.linspace(-4, 4, 37).reshape(1, 37)
    comp = _comp(fn)
    rt = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", seed=7)
    rows = rt.evaluate_computation(comp, {"x": x})["output_0"]
    monkeypatch.setattr(fxp, "_rows_ok", lambda sess, x: False)
    rt2 = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", seed=7)
    generic = rt2.evaluate_computation(comp, {"x": x})["output_0"]
    np.testing.assert_array_equal(rows, generic)
    np.testing.assert_allclose(rows, ref(x), rtol=2e-3, atol=2e-4)
