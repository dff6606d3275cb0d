"""Data-parallel replicas of the 3-party session (SURVEY §2.7 DP; BASELINE config 5):
R x 3 worker processes (gloo here, RCCL on GPUs), batch-sharded inputs, per-replica
process groups for the protocol messages, and an all-gather of the revealed outputs
across the replicas' output owners."""
import numpy as np
import pytest

import moose_amd as pm
from moose_amd.parallel.replicas import shard_arguments
from moose_amd.runtime.distributed import DistributedMooseRuntime
from moose_amd.runtime.local import LocalMooseRuntime

IDS = ["alice", "bob", "carole"]


def _logreg_inference():
    alice, bob, carole = (pm.host_placement(n) for n in IDS)
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(14, 23)

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64)),
          w: pm.Argument(placement=bob, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fx)
        with bob:
            wf = pm.cast(w, dtype=fx)
        with rep:
            y = pm.sigmoid(pm.dot(xf, wf))
            c = pm.less(pm.dot(xf, wf), pm.constant(np.array(0.0), dtype=fx))
        with carole:
            out = pm.cast(y, dtype=pm.float64)
            neg = pm.identity(c)
        return out, neg

    return f


def test_shard_arguments_splits_rows_and_replicates_rest():
    x = np.arange(22).reshape(11, 2)
    parts = shard_arguments({"x": x, "w": 5}, ["x"], 3)
    assert [p["x"].shape[0] for p in parts] == [4, 4, 3]
    np.testing.assert_array_equal(np.concatenate([p["x"] for p in parts]), x)
    assert all(p["w"] == 5 for p in parts)
    with pytest.raises(KeyError):
        shard_arguments({"x": x}, ["y"], 2)
    with pytest.raises(ValueError):
        shard_arguments({"x": np.ones((1, 3))}, ["x"], 2)


@pytest.mark.parametrize("replicas", [2])
def test_replicated_sessions_match_single_session(replicas):
    rng = np.random.default_rng(0)
    x, w = rng.uniform(-1, 1, (11, 6)), rng.uniform(-1, 1, (6, 2))
    f = _logreg_inference()
    rt = DistributedMooseRuntime(IDS, backend="gloo", replicas=replicas, shard_args=["x"],
                                 timeout=300)
    got = rt.evaluate_computation(f, {"x": x, "w": w})
    ref = LocalMooseRuntime(IDS, device="cpu").evaluate_computation(f, {"x": x, "w": w})
    assert got["output_0"].shape == (11, 2)
    np.testing.assert_allclose(got["output_0"], 1 / (1 + np.exp(-(x @ w))), atol=1e-4)
    np.testing.assert_allclose(got["output_0"], ref["output_0"], atol=1e-4)
    np.testing.assert_array_equal(np.asarray(got["output_1"]).astype(bool), (x @ w) < 0)
    assert set(rt.last_timings) == set(IDS)
