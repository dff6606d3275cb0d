"""Intra-party dataflow lanes (runtime/lanes.py): the static chain plan on the host, and on
the GPU bitwise-identical results with 1 and 4 lanes -- eagerly and under hipGraph capture
-- for a computation with independent branches (reference: independent operations run as
concurrent tasks, execution/asynchronous.rs:456-530)."""
import numpy as np
import pytest

import moose_amd as pm
from moose_amd.ir.computation import Computation
from moose_amd.runtime.lanes import LanePlan


def test_plan_chains_follow_dependencies():
    src = """a = Constant{value = HostFloat64Tensor([1.0])}: () -> HostFloat64Tensor () @Host(alice)
b = Constant{value = HostFloat64Tensor([2.0])}: () -> HostFloat64Tensor () @Host(alice)
c = Add: (HostFloat64Tensor, HostFloat64Tensor) -> HostFloat64Tensor (a, a) @Host(alice)
d = Add: (HostFloat64Tensor, HostFloat64Tensor) -> HostFloat64Tensor (b, b) @Host(alice)
e = Add: (HostFloat64Tensor, HostFloat64Tensor) -> HostFloat64Tensor (c, d) @Host(alice)
"""
    ops = Computation.from_textual(src).toposorted().operations
    plan = LanePlan(ops, 4)
    ln = plan.lane
    assert ln["a"] != ln["b"]  # independent roots start separate chains
    assert ln["c"] == ln["a"] and ln["d"] == ln["b"]  # each chain extends its tail
    assert ln["e"] in (ln["c"], ln["d"])  # the join continues one of them
    # exactly the value coming from the other chain needs an event
    other = "d" if ln["e"] == ln["c"] else "c"
    assert plan.crosses(other, ln[other]) and not plan.crosses("a", ln["a"])
    assert plan.width() == 2
    assert set(LanePlan(ops, 1).lane.values()) == {0}


def _wide_comp(branches=4, n=64, k=10):
    alice, bob, carole = (pm.host_placement(x) for x in ("alice", "bob", "carole"))
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(24, 40)
    rng = np.random.default_rng(3)
    ws = [rng.normal(size=(k, 1)) * 0.3 for _ in range(branches)]

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fx)
        wf = []
        with bob:
            for w in ws:
                wf.append(pm.cast(pm.constant(w, dtype=pm.float64), dtype=fx))
        with rep:
            ys = [pm.sigmoid(pm.dot(xf, w)) for w in wf]
            acc = ys[0]
            for y in ys[1:]:
                acc = pm.add(acc, y)
        with carole:
            out = pm.cast(acc, dtype=pm.float64)
        return out

    x = rng.normal(size=(n, k))
    ref = sum(1 / (1 + np.exp(-(x @ w))) for w in ws)
    return f, x, ref


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [False, True])
def test_lanes_match_single_stream_bitwise(graphs):
    f, x, ref = _wide_comp()
    outs = {}
    for lanes in (1, 4):
        rt = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", seed=11,
                                  use_graphs=graphs, lanes=lanes)
        for _ in range(3 if graphs else 1):  # graphs: warm-up, capture, replays
            r = rt.evaluate_computation(f, {"x": x})
        if graphs:
            assert rt._graphs.plans, getattr(rt._graphs, "last_error", "capture failed")
        outs[lanes] = np.asarray(list(r.values())[0])
        np.testing.assert_allclose(outs[lanes], ref, atol=1e-4)
    if not graphs:  # same seed, same program order of PRF draws -> identical shares
        np.testing.assert_array_equal(outs[1], outs[4])


def test_batched_ops_only_read_values_ordered_on_their_lane():
    """A Dot executed ahead of its turn (batched into an earlier Dot's launch) runs on the
    earlier Dot's lane: its operands must be produced there, before the fork, or already
    waited on (no event existed for a same-lane producer of a later Dot)."""
    from moose_amd.runtime.lanes import LaneRunner

    r = LaneRunner("cpu", 2)
    r.cur = 0
    r.where = {"w0": 0, "w1": 1, "x": 0}
    r.waited = [set(), set()]
    assert r.ordered_here(["x", "w0"])
    assert r.ordered_here(["arg"])          # produced before the lanes forked
    assert not r.ordered_here(["x", "w1"])  # lane 1's value, never waited on by lane 0
    r.waited[0].add("w1")
    assert r.ordered_here(["x", "w1"])


@pytest.mark.gpu
def test_lanes_slow_producer_on_other_lane():
    """Weights of later Dots come from long chains on other lanes; the result must match
    the single-stream run however the lanes interleave."""
    alice, bob, carole = (pm.host_placement(x) for x in ("alice", "bob", "carole"))
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(24, 40)
    rng = np.random.default_rng(4)
    ws = [rng.normal(size=(512, 256)) * 0.05 for _ in range(4)]

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fx)
        wf = []
        with bob:
            for i, w in enumerate(ws):
                c = pm.constant(w, dtype=pm.float64)
                for _ in range(8 * i):  # slower producers for later branches
                    c = pm.add(c, pm.constant(np.zeros_like(w), dtype=pm.float64))
                wf.append(pm.cast(c, dtype=fx))
        with rep:
            ys = [pm.dot(xf, w) for w in wf]
            acc = ys[0]
            for y in ys[1:]:
                acc = pm.add(acc, y)
        with carole:
            return pm.cast(acc, dtype=pm.float64)

    x = rng.normal(size=(256, 512)) * 0.05
    outs = {}
    for lanes in (1, 4):
        rt = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", seed=5,
                                  lanes=lanes)
        outs[lanes] = np.asarray(list(rt.evaluate_computation(f, {"x": x}).values())[0])
    np.testing.assert_allclose(outs[1], sum(x @ w for w in ws), atol=1e-6)
    # (batching may differ between the runs, and with it the TruncPr rounding: 1 ulp)
    np.testing.assert_allclose(outs[1], outs[4], atol=1e-9)
