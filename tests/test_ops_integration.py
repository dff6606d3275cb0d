"""Per-operator end-to-end tests through the eDSL + LocalMooseRuntime, on host,
replicated and mirrored placements, against numpy (the coverage of the reference's
``pymoose/rust_integration_tests``: add_n, argmax, boolean ops, concat, dtype
conversions, exp, log, maximum, mirrored ops, ones/zeros, reduce max, relu, reshape,
select, shape, sigmoid, slicing, softmax, sqrt, squeeze, transpose, uint64, save/load)."""
import numpy as np
import pytest

import moose_amd as pm
from moose_amd.runtime.local import LocalMooseRuntime

FP = pm.fixed(14, 23)
ALICE, BOB, CAROLE = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
REP = pm.replicated_placement("rep", players=[ALICE, BOB, CAROLE])
MIR = pm.mirrored_placement("mir", players=[ALICE, BOB, CAROLE])
IDS = ["alice", "bob", "carole"]


def run(comp, args=None, **kw):
    rt = LocalMooseRuntime(IDS, device="cpu", **kw)
    out = rt.evaluate_computation(comp, args or {})
    return rt, out


def only(out):
    assert len(out) == 1
    return np.asarray(list(out.values())[0])


# ---------------------------------------------------------------------------
# dtype conversions (host)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("x,src,dst", [
    ([-1.0, 0, 1, 2], pm.float64, pm.float32),
    ([-1.0, 0, 1, 2], pm.float32, pm.float64),
    ([-1.0, 0, 1, 2], pm.float64, pm.bool_),
    ([1, 0, 1, 1], pm.bool_, pm.float64),
    ([3.0, 0, 1, 2], pm.float64, pm.uint64),
    ([3, 0, 1, 2], pm.uint64, pm.float64),
    ([3, 0, 1, 2], pm.uint64, pm.bool_),
    ([1, 0, 1, 1], pm.bool_, pm.uint64),
    ([-1.5, 0.25, 3.0], pm.float64, FP),
    ([-1.5, 0.25, 3.0], pm.float32, pm.fixed(24, 40)),
])
def test_dtype_conversions(x, src, dst):
    @pm.computation
    def f():
        with ALICE:
            c = pm.constant(np.array(x), dtype=src)
            y = pm.cast(c, dtype=dst)
            return pm.save("x", y)

    rt, _ = run(f)
    got = np.asarray(rt.read_value_from_storage("alice", "x"))
    want = np.array(x).astype(src.numpy_dtype if hasattr(src, "numpy_dtype") else None)
    if dst.is_fixedpoint:
        np.testing.assert_allclose(got, np.array(x, dtype=np.float64), atol=1e-6)
    elif dst == pm.bool_:
        np.testing.assert_array_equal(got.astype(bool), np.array(x) != 0)
    else:
        np.testing.assert_allclose(got.astype(np.float64), np.asarray(want, dtype=np.float64))


# ---------------------------------------------------------------------------
# unary math on host and replicated
# ---------------------------------------------------------------------------
_UNARY = {
    "exp": (pm.exp, np.exp, [-2.0, -0.5, 0.0, 1.0, 3.0], 1e-3),
    "sigmoid": (pm.sigmoid, lambda v: 1 / (1 + np.exp(-v)), [-4.0, -1.0, 0.0, 0.5, 6.0], 1e-3),
    "relu": (pm.relu, lambda v: np.maximum(v, 0), [-4.0, -1.0, 0.0, 0.5, 6.0], 1e-6),
    "abs": (pm.abs, np.abs, [-4.0, -1.0, 0.0, 0.5, 6.0], 1e-6),
    "log": (pm.log, np.log, [0.1, 0.5, 1.0, 2.0, 100.0], 1e-3),
    "log2": (pm.log2, np.log2, [0.1, 0.5, 1.0, 2.0, 100.0], 1e-3),
    "sqrt": (pm.sqrt, np.sqrt, [0.1, 0.5, 1.0, 2.0, 100.0], 2e-3),
}


@pytest.mark.parametrize("name", sorted(_UNARY))
@pytest.mark.parametrize("where", ["host", "rep"])
def test_unary(name, where):
    op, ref, xs, tol = _UNARY[name]
    plc = ALICE if where == "host" else REP

    @pm.computation
    def f(x: pm.Argument(ALICE, vtype=pm.TensorType(pm.float64))):
        with ALICE:
            xf = pm.cast(x, dtype=FP) if where == "rep" else x
        with plc:
            y = op(xf)
        with BOB:
            return pm.cast(y, dtype=pm.float64) if where == "rep" else pm.identity(y)

    _, out = run(f, {"x": np.array(xs)})
    np.testing.assert_allclose(only(out), ref(np.array(xs)), rtol=tol, atol=tol)


@pytest.mark.parametrize("where", ["host", "rep"])
def test_softmax_argmax_maximum(where):
    x = np.array([[1.0, -2.0, 0.5], [0.0, 3.0, -1.0]])
    plc = ALICE if where == "host" else REP

    @pm.computation
    def f(a: pm.Argument(ALICE, vtype=pm.TensorType(pm.float64))):
        with ALICE:
            af = pm.cast(a, dtype=FP) if where == "rep" else a
        with plc:
            sm = pm.softmax(af, axis=1, upmost_index=3)
            am = pm.argmax(af, axis=1, upmost_index=3)
            mx = pm.maximum([pm.index_axis(af, 1, i) for i in range(3)])
        with BOB:
            cast = (lambda v: pm.cast(v, dtype=pm.float64)) if where == "rep" else pm.identity
            return cast(sm), pm.identity(am), cast(mx)

    _, out = run(f, {"a": x})
    e = np.exp(x - x.max(1, keepdims=True))
    np.testing.assert_allclose(out["output_0"], e / e.sum(1, keepdims=True), atol=2e-3)
    np.testing.assert_array_equal(np.asarray(out["output_1"]).astype(np.int64), x.argmax(1))
    np.testing.assert_allclose(out["output_2"], x.max(1), atol=1e-6)


# ---------------------------------------------------------------------------
# arithmetic, add_n, comparisons, mux, boolean ops
# ---------------------------------------------------------------------------
def test_add_n_mul_div_dot_rep():
    x = np.array([[1.5, -2.0], [0.25, 3.0]])

    @pm.computation
    def f(a: pm.Argument(ALICE, vtype=pm.TensorType(pm.float64)),
          b: pm.Argument(BOB, vtype=pm.TensorType(pm.float64))):
        with ALICE:
            af = pm.cast(a, dtype=FP)
        with BOB:
            bf = pm.cast(b, dtype=FP)
        with REP:
            s = pm.add_n([af, bf, af])
            m = pm.mul(af, bf)
            d = pm.div(af, bf)
            p = pm.dot(af, bf)
            q = pm.sub(af, bf)
        with CAROLE:
            return tuple(pm.cast(v, dtype=pm.float64) for v in (s, m, d, p, q))

    _, out = run(f, {"a": x, "b": x + 2.5})
    y = x + 2.5
    np.testing.assert_allclose(out["output_0"], 2 * x + y, atol=1e-5)
    np.testing.assert_allclose(out["output_1"], x * y, atol=1e-5)
    np.testing.assert_allclose(out["output_2"], x / y, atol=1e-3)
    np.testing.assert_allclose(out["output_3"], x @ y, atol=1e-5)
    np.testing.assert_allclose(out["output_4"], x - y, atol=1e-5)


@pytest.mark.parametrize("where", ["host", "rep"])
def test_comparisons_mux_and_boolean_ops(where):
    x = np.array([1.0, -2.0, 3.0, 0.5])
    y = np.array([0.0, -1.0, 3.5, 0.5])
    plc = ALICE if where == "host" else REP

    @pm.computation
    def f(a: pm.Argument(ALICE, vtype=pm.TensorType(pm.float64)),
          b: pm.Argument(BOB, vtype=pm.TensorType(pm.float64))):
        with ALICE:
            af = pm.cast(a, dtype=FP)
        with BOB:
            bf = pm.cast(b, dtype=FP)
        with plc:
            lt = pm.less(af, bf)
            gt = pm.greater(af, bf)
            both = pm.logical_and(lt, gt)
            either = pm.logical_or(lt, gt)
        with REP:  # mux is a replicated-placement operation (as in pymoose)
            mx = pm.mux(lt, bf, af)
        with CAROLE:
            return (pm.identity(lt), pm.identity(gt), pm.identity(both), pm.identity(either),
                    pm.cast(mx, dtype=pm.float64))

    _, out = run(f, {"a": x, "b": y})
    np.testing.assert_array_equal(np.asarray(out["output_0"]).astype(bool), x < y)
    np.testing.assert_array_equal(np.asarray(out["output_1"]).astype(bool), x > y)
    np.testing.assert_array_equal(np.asarray(out["output_2"]).astype(bool), (x < y) & (x > y))
    np.testing.assert_array_equal(np.asarray(out["output_3"]).astype(bool), (x < y) | (x > y))
    np.testing.assert_allclose(out["output_4"], np.maximum(x, y), atol=1e-6)


def test_boolean_inputs_on_rep():
    a = np.array([True, False, True, False])
    b = np.array([True, True, False, False])

    @pm.computation
    def f(x: pm.Argument(ALICE, vtype=pm.TensorType(pm.bool_)),
          y: pm.Argument(BOB, vtype=pm.TensorType(pm.bool_))):
        with REP:
            z = pm.logical_and(x, y)
            w = pm.logical_or(x, y)
        with CAROLE:
            return pm.identity(z), pm.identity(w)

    _, out = run(f, {"x": a, "y": b})
    np.testing.assert_array_equal(np.asarray(out["output_0"]).astype(bool), a & b)
    np.testing.assert_array_equal(np.asarray(out["output_1"]).astype(bool), a | b)


def test_uint64_on_rep():
    a = np.array([1, 2, 3, 2**40], dtype=np.uint64)
    b = np.array([7, 0, 5, 3], dtype=np.uint64)

    @pm.computation
    def f(x: pm.Argument(ALICE, vtype=pm.TensorType(pm.uint64)),
          y: pm.Argument(BOB, vtype=pm.TensorType(pm.uint64))):
        with REP:
            s = pm.add(x, y)
        with CAROLE:
            return pm.identity(s)

    _, out = run(f, {"x": a, "y": b})
    np.testing.assert_array_equal(np.asarray(out["output_0"]).astype(np.uint64), a + b)


# ---------------------------------------------------------------------------
# shape ops on host and replicated
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("where", ["host", "rep"])
def test_shape_ops(where):
    x = np.arange(24, dtype=np.float64).reshape(2, 3, 4) / 4
    plc = ALICE if where == "host" else REP

    @pm.computation
    def f(a: pm.Argument(ALICE, vtype=pm.TensorType(pm.float64))):
        with ALICE:
            af = pm.cast(a, dtype=FP)
        with plc:
            r = pm.reshape(af, [6, 4])
            t = pm.transpose(r)
            e = pm.expand_dims(af, 0)
            s = pm.squeeze(e, 0)
            i = pm.index_axis(af, axis=2, index=1)
            c = pm.concatenate([af, af], axis=1)
            sl = af[0:1, 1:3]
        with CAROLE:
            return tuple(pm.cast(v, dtype=pm.float64) for v in (r, t, s, i, c, sl))

    _, out = run(f, {"a": x})
    np.testing.assert_allclose(out["output_0"], x.reshape(6, 4))
    np.testing.assert_allclose(out["output_1"], x.reshape(6, 4).T)
    np.testing.assert_allclose(out["output_2"], x)
    np.testing.assert_allclose(out["output_3"], x[:, :, 1])
    np.testing.assert_allclose(out["output_4"], np.concatenate([x, x], axis=1))
    np.testing.assert_allclose(out["output_5"], x[0:1, 1:3])


def test_shape_ones_zeros_and_sum_mean():
    x = np.arange(6, dtype=np.float64).reshape(2, 3)

    @pm.computation
    def f(a: pm.Argument(ALICE, vtype=pm.TensorType(pm.float64))):
        with ALICE:
            af = pm.cast(a, dtype=FP)
        with REP:
            shp = pm.shape(af)
            o = pm.ones(shp, dtype=pm.float64)
            s0 = pm.sum(af, axis=0)
            mn = pm.mean(af, axis=1)
        with BOB:
            z = pm.zeros(shp, dtype=pm.float64)
            return (pm.identity(o), pm.identity(z), pm.cast(s0, dtype=pm.float64),
                    pm.cast(mn, dtype=pm.float64))

    _, out = run(f, {"a": x})
    np.testing.assert_allclose(out["output_0"], np.ones((2, 3)))
    np.testing.assert_allclose(out["output_1"], np.zeros((2, 3)))
    np.testing.assert_allclose(out["output_2"], x.sum(0), atol=1e-6)
    np.testing.assert_allclose(out["output_3"], x.mean(1), atol=1e-5)


def test_select_and_strided_slices_host():
    x = np.arange(12, dtype=np.float64).reshape(3, 4)
    mask = np.array([True, False, True])

    @pm.computation
    def f(a: pm.Argument(ALICE, vtype=pm.TensorType(pm.float64)),
          m: pm.Argument(ALICE, vtype=pm.TensorType(pm.bool_))):
        with ALICE:
            s = pm.select(a, axis=0, index=m)
            st = a[::2, 1:]
        with BOB:
            return pm.identity(s), pm.identity(st)

    _, out = run(f, {"a": x, "m": mask})
    np.testing.assert_allclose(out["output_0"], x[mask])
    np.testing.assert_allclose(out["output_1"], x[::2, 1:])


# ---------------------------------------------------------------------------
# mirrored placement, save/load, identity returns
# ---------------------------------------------------------------------------
def test_mirrored_constants_with_replicated():
    x = np.array([1.0, -2.0, 0.5])

    @pm.computation
    def f(a: pm.Argument(ALICE, vtype=pm.TensorType(pm.float64))):
        with ALICE:
            af = pm.cast(a, dtype=FP)
        with MIR:
            c = pm.cast(pm.constant(np.array([2.0, 3.0, -1.0])), dtype=FP)
        with REP:
            y = pm.mul(af, c)
            z = pm.add(y, c)
        with BOB:
            return pm.cast(z, dtype=pm.float64)

    _, out = run(f, {"a": x})
    np.testing.assert_allclose(only(out), x * [2, 3, -1] + [2, 3, -1], atol=1e-6)


def test_save_load_roundtrip_and_storage():
    @pm.computation
    def f():
        with ALICE:
            v = pm.load("input_key", dtype=pm.float64)
            w = pm.add(v, v)
            return pm.save("result", w)

    rt = LocalMooseRuntime(IDS, storage_mapping={"alice": {"input_key": np.array([1.0, 2.5])}},
                           device="cpu")
    rt.evaluate_computation(f, {})
    np.testing.assert_allclose(rt.read_value_from_storage("alice", "result"), [2.0, 5.0])


@pytest.mark.parametrize("ring", [64, 128])
def test_fixedpoint_ring_option(ring):
    x = np.array([1.25, -3.5])

    @pm.computation
    def f(a: pm.Argument(ALICE, vtype=pm.TensorType(pm.float64))):
        with ALICE:
            af = pm.cast(a, dtype=FP)
        with REP:
            y = pm.mul(af, af)
        with BOB:
            return pm.cast(y, dtype=pm.float64)

    _, out = run(f, {"a": x}, fixedpoint_ring=ring)
    np.testing.assert_allclose(only(out), x * x, atol=1e-5)
