"""Intra-evaluation overlap for the per-party sessions (runtime/interpreter.py
Interpreter._merge_unary): independent multi-round elementwise ops of one kind, placement
and dtype run as ONE protocol run over their concatenated inputs, so k independent chains
cost the message rounds of one.  On by default for SPMD processes and in-process parties;
the values are those of the ops run one by one up to TruncPr's rounding draws."""
import numpy as np
import pytest

import moose_amd as pm
from moose_amd.runtime import interpreter as I
from moose_amd.runtime.distributed import DistributedMooseRuntime
from moose_amd.runtime.local import LocalMooseRuntime

IDS = ["alice", "bob", "carole"]


def _comp(src="alice"):
    alice, bob, carole = (pm.host_placement(n) for n in IDS)
    owner = pm.host_placement(src)
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(24, 40)

    @pm.computation
    def f(x: pm.Argument(placement=owner, vtype=pm.TensorType(pm.float64)),
          y: pm.Argument(placement=bob, vtype=pm.TensorType(pm.float64))):
        with owner:
            xf = pm.cast(x, dtype=fx)
        with bob:
            yf = pm.cast(y, dtype=fx)
        with rep:
            a = pm.sigmoid(xf)
            b = pm.sigmoid(yf)
            c = pm.exp(xf)
            d = pm.exp(yf)
        with carole:
            return (pm.cast(a, dtype=pm.float64), pm.cast(b, dtype=pm.float64),
                    pm.cast(c, dtype=pm.float64), pm.cast(d, dtype=pm.float64))

    return f


def _args():
    return {"x": np.linspace(-6, 3, 12).reshape(3, 4), "y": np.linspace(-3, 2, 10)}


def _check(out, args):
    x, y = args["x"], args["y"]
    refs = [1 / (1 + np.exp(-x)), 1 / (1 + np.exp(-y)), np.exp(x), np.exp(y)]
    vals = [np.asarray(v, dtype=np.float64) for v in out.values()]
    for v in vals:
        err = min(np.abs(v - w).max() / max(1.0, np.abs(w).max()) for w in refs
                  if w.shape == v.shape)
        assert err < 1e-6


def test_independent_chains_share_rounds(monkeypatch):
    args = _args()
    monkeypatch.setattr(I, "MERGE_ROUNDS", False)
    rt = LocalMooseRuntime(IDS, device_map={i: "cpu" for i in IDS}, seed=3)
    _check(rt.evaluate_computation(_comp(), args), args)
    serial = rt.last_stats.rounds
    monkeypatch.setattr(I, "MERGE_ROUNDS", True)
    rt = LocalMooseRuntime(IDS, device_map={i: "cpu" for i in IDS}, seed=3)
    _check(rt.evaluate_computation(_comp(), args), args)
    merged = rt.last_stats.rounds
    # two sigmoids and two exps: each pair costs the rounds of one
    assert merged <= serial // 2 + 4, (merged, serial)


def test_merged_chains_across_processes_with_an_outsider():
    """SPMD processes over gloo, the input owned by a host outside the placement: every
    process forms the same groups from the computation's structure alone."""
    idents = IDS + ["dave"]
    args = _args()
    comp = _comp(src="dave")
    local = LocalMooseRuntime(idents, device="cpu", seed=1).evaluate_computation(comp, args)
    got = DistributedMooseRuntime(idents, backend="gloo", seed=1,
                                  timeout=300).evaluate_computation(comp, args)
    assert set(got) == set(local)
    for k in local:
        np.testing.assert_allclose(np.asarray(got[k], dtype=np.float64),
                                   np.asarray(local[k], dtype=np.float64), atol=1e-6)
    _check(got, args)


@pytest.mark.gpu
def test_merged_chains_graph_replays_bitwise_equal_eager():
    args = _args()
    comp = _comp()
    devs = {i: "cuda:0" for i in IDS}
    want = LocalMooseRuntime(IDS, device_map=devs, seed=11,
                             use_graphs=False).evaluate_computation(comp, args)
    rt = LocalMooseRuntime(IDS, device_map=devs, seed=11, use_graphs=True)
    for _ in range(4):
        got = rt.evaluate_computation(comp, args)
        for k in want:
            assert np.array_equal(np.asarray(got[k]), np.asarray(want[k])), k
    _check(got, args)
