"""End-to-end runtimes on the MI355X: the logical interpreter (stacked session) and the
lowered host graph both run their ring kernels on the GPU and agree with the CPU run."""
import numpy as np
import pytest

import moose_amd as pm
from moose_amd.compiler import passes
from moose_amd.ops import native as nat
from moose_amd.runtime.local import LocalMooseRuntime

pytestmark = pytest.mark.gpu


def _comp():
    fp = pm.fixed(14, 23)
    alice, bob, carole = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64)),
          y: pm.Argument(placement=bob, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fp)
        with bob:
            yf = pm.cast(y, dtype=fp)
        with rep:
            z = pm.dot(xf, yf)
            s = pm.sigmoid(z)
            e = pm.exp(z)
            sm = pm.softmax(z, axis=1, upmost_index=8)
            am = pm.argmax(z, axis=1, upmost_index=8)
            lg = pm.log(pm.add(e, e))
        with carole:
            return (pm.cast(z, dtype=pm.float64), pm.cast(s, dtype=pm.float64),
                    pm.cast(sm, dtype=pm.float64), pm.identity(am), pm.cast(lg, dtype=pm.float64))

    return f


@pytest.fixture(scope="module")
def args():
    # |z| stays well inside fixed(14, 23)'s integral range for exp/log (2 e^z < 2^14)
    rng = np.random.default_rng(5)
    return {"x": rng.uniform(-0.5, 0.5, (64, 96)), "y": rng.uniform(-1, 1, (96, 8))}


@pytest.mark.parametrize("ring", [64, 128])
def test_interpreter_gpu_matches_cpu(args, ring):
    f = _comp()
    gpu = LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", fixedpoint_ring=ring)
    cpu = LocalMooseRuntime(["alice", "bob", "carole"], device="cpu", fixedpoint_ring=ring)
    a, b = gpu.evaluate_computation(f, args), cpu.evaluate_computation(f, args)
    assert nat.loaded_path().endswith("libmoosex.so")
    z = args["x"] @ args["y"]
    np.testing.assert_allclose(a["output_0"], z, atol=1e-4)
    np.testing.assert_allclose(a["output_1"], 1 / (1 + np.exp(-z)), atol=1e-3)
    e = np.exp(z - z.max(axis=1, keepdims=True))
    np.testing.assert_allclose(a["output_2"], e / e.sum(axis=1, keepdims=True), atol=2e-3)
    assert (np.asarray(a["output_3"]) == z.argmax(axis=1)).mean() > 0.95
    np.testing.assert_allclose(a["output_4"], np.log(2 * np.exp(z)), atol=5e-3)
    for k in a:
        np.testing.assert_allclose(np.asarray(a[k], dtype=float), np.asarray(b[k], dtype=float),
                                   atol=5e-3)


def test_lowered_graph_on_gpu(args):
    f = _comp()
    rt = LocalMooseRuntime(["alice", "bob", "carole"], device="cuda")
    ref = rt.evaluate_computation(f, args)
    got = rt.evaluate_computation(f, args, compiler_passes=passes.DEFAULT_PASSES)
    for k in ref:
        np.testing.assert_allclose(np.asarray(got[k], dtype=float), np.asarray(ref[k], dtype=float),
                                   atol=5e-3)


@pytest.mark.parametrize("shapes", [((300, 260), (260,)), ((260,), (260, 300)), ((64, 96), (96,))])
def test_secret_matrix_vector_dot(shapes):
    """Secret matrix . secret vector (and vector . matrix) at fixed(24, 40): the stacked
    right operand is [3, K], which the rolled-pair CRT GEMM must decline."""
    fp = pm.fixed(24, 40)
    alice, bob, carole = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64)),
          y: pm.Argument(placement=bob, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fp)
        with bob:
            yf = pm.cast(y, dtype=fp)
        with rep:
            z = pm.dot(xf, yf)
        with carole:
            return pm.cast(z, dtype=pm.float64)

    rng = np.random.default_rng(11)
    x, y = rng.uniform(-1, 1, shapes[0]), rng.uniform(-1, 1, shapes[1])
    rt = LocalMooseRuntime(["alice", "bob", "carole"], device="cuda")
    got = rt.evaluate_computation(f, {"x": x, "y": y})["output_0"]
    np.testing.assert_allclose(got, x @ y, atol=1e-6)
