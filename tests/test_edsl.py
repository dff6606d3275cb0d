"""eDSL tracing: the traced computation's operations, inputs and signatures (reference
``pymoose/pymoose/edsl/base_test.py``), serde round trips and conversion to the native
IR."""
import numpy as np
import pytest

from moose_amd.computation import dtypes
from moose_amd.computation import operations as ops
from moose_amd.computation import types as ty
from moose_amd.computation import utils
from moose_amd.edsl import base as edsl
from moose_amd.edsl.tracer import trace

F64 = ty.TensorType(dtypes.float64)


def _sig(args, ret):
    return ops.OpSignature(args, ret)


@pytest.mark.parametrize("fn,cls,name", [
    (lambda x, y: x + y, ops.AddOperation, "add"),
    (lambda x, y: x - y, ops.SubOperation, "sub"),
    (lambda x, y: x * y, ops.MulOperation, "mul"),
    (lambda x, y: x / y, ops.DivOperation, "div"),
    (lambda x, y: x @ y, ops.DotOperation, "dot"),
    (lambda x, y: x > y, ops.GreaterOperation, "greater"),
    (lambda x, y: x < y, ops.LessOperation, "less"),
])
def test_binary_dunders(fn, cls, name):
    alice = edsl.host_placement("alice")

    @edsl.computation
    def comp():
        with alice:
            x = edsl.constant(np.array([1.0, 2.0, 3.0]))
            return fn(x, x)

    op = trace(comp).operation(f"{name}_0")
    out = ty.TensorType(dtypes.bool_) if name in ("less", "greater") else F64
    assert op == cls(placement_name="alice", name=f"{name}_0",
                     inputs={"lhs": "constant_0", "rhs": "constant_0"},
                     signature=_sig({"lhs": F64, "rhs": F64}, out))


def test_abs_neg_identity():
    alice, bob = edsl.host_placement("alice"), edsl.host_placement("bob")

    @edsl.computation
    def comp():
        with alice:
            x = edsl.constant(np.array([1.0, -2.0]))
            a = abs(x)
        with bob:
            return edsl.identity(a)

    c = trace(comp)
    assert c.operation("abs_0") == ops.AbsOperation(
        placement_name="alice", name="abs_0", inputs={"x": "constant_0"},
        signature=_sig({"x": F64}, F64))
    assert c.operation("identity_0").placement_name == "bob"


def test_concatenate_add_n_and_reductions():
    p0 = edsl.host_placement("p0")

    @edsl.computation
    def comp():
        with p0:
            a = edsl.constant(np.array([1.0]))
            b = edsl.constant(np.array([2.0]))
            c = edsl.concatenate([a, b])
            s = edsl.add_n([a, b, a])
            m = edsl.sum(c, axis=0)
            n = edsl.mean(c)
            return c, s, m, n

    t = trace(comp)
    cat = t.operation("concatenate_0")
    assert cat.inputs == {"array0": "constant_0", "array1": "constant_1"} and cat.axis == 0
    assert t.operation("add_n_0").inputs == {"array0": "constant_0", "array1": "constant_1",
                                             "array2": "constant_0"}
    assert t.operation("sum_0").axis == 0 and t.operation("mean_0").axis is None


def test_shape_ops_and_attributes():
    p0 = edsl.host_placement("p0")

    @edsl.computation
    def comp():
        with p0:
            x = edsl.constant(np.ones((2, 3)))
            r = edsl.reshape(x, [3, 2])
            t = edsl.transpose(r)
            e = edsl.expand_dims(t, [0])
            s = edsl.squeeze(e, 0)
            i = edsl.index_axis(s, axis=1, index=1)
            a = edsl.atleast_2d(i, to_column_vector=True)
            return a

    c = trace(comp)
    kinds = [type(op).__name__ for op in c.operations.values()]
    for k in ("ReshapeOperation", "TransposeOperation", "ExpandDimsOperation",
              "SqueezeOperation", "IndexAxisOperation", "AtLeast2DOperation"):
        assert k in kinds
    assert c.operation("index_axis_0").axis == 1 and c.operation("index_axis_0").index == 1
    assert c.operation("atleast_2d_0").to_column_vector is True


def test_ones_zeros_and_mux_on_replicated():
    alice, bob, carole = (edsl.host_placement(n) for n in ("alice", "bob", "carole"))
    rep = edsl.replicated_placement("rep", [alice, bob, carole])
    fx = dtypes.fixed(14, 23)

    @edsl.computation
    def comp(x: edsl.Argument(alice, vtype=ty.TensorType(fx))):
        with rep:
            sel = edsl.less(x, x)
            y = edsl.mux(sel, x, x)
        with bob:
            o = edsl.ones(edsl.shape(x), dtype=dtypes.float64)
            z = edsl.zeros(edsl.shape(x), dtype=dtypes.float64)
        return y, o, z

    c = trace(comp)
    mux = c.operation("mux_0")
    assert mux.placement_name == "rep" and set(mux.inputs) == {"selector", "x", "y"}
    assert c.operation("ones_0").placement_name == "bob"


def test_mux_requires_replicated_placement():
    alice = edsl.host_placement("alice")
    fx = dtypes.fixed(14, 23)

    @edsl.computation
    def comp(x: edsl.Argument(alice, vtype=ty.TensorType(fx))):
        with alice:
            return edsl.mux(edsl.less(x, x), x, x)

    with pytest.raises(AssertionError):
        trace(comp)


def test_constant_load_and_tensor_arguments():
    alice = edsl.host_placement("alice")

    @edsl.computation
    def comp(x: edsl.Argument(alice, dtype=dtypes.uint64)):
        with alice:
            y = edsl.load("key", dtype=dtypes.float64)
            z = edsl.load("key2", query="q", dtype=dtypes.float64)
            return x, y, z

    c = trace(comp)
    assert c.operation("x").return_type == ty.TensorType(dtypes.uint64)
    load = c.operation("load_0")
    assert load.inputs["key"].startswith("constant") and "query" in load.inputs


@pytest.mark.parametrize("src,dst", [(dtypes.float64, dtypes.fixed(14, 23)),
                                     (dtypes.fixed(14, 23), dtypes.float64),
                                     (dtypes.float64, dtypes.float32)])
def test_cast(src, dst):
    alice = edsl.host_placement("alice")

    @edsl.computation
    def comp():
        with alice:
            x = edsl.constant(np.array([1.0]), dtype=src)
            return edsl.cast(x, dtype=dst)

    c = trace(comp)
    casts = [op for op in c.operations.values() if isinstance(op, ops.CastOperation)]
    assert casts[-1].signature.return_type == ty.TensorType(dst)


def test_role_map_and_tagged_outputs():
    alice, bob = edsl.host_placement("alice"), edsl.host_placement("bob")

    @edsl.computation(role_map={"alice": "carole"})
    def comp():
        with alice:
            x = edsl.constant(np.array([1.0]))
        with bob:
            y = edsl.identity(x)
            return edsl.output("tagged", y)

    c = trace(comp)
    assert "carole" in c.placements and "alice" not in c.placements
    outs = [op for op in c.operations.values() if isinstance(op, ops.OutputOperation)]
    assert [o.tag for o in outs] == ["tagged"]


def test_msgpack_serde_roundtrip_and_native_conversion():
    alice, bob, carole = (edsl.host_placement(n) for n in ("alice", "bob", "carole"))
    rep = edsl.replicated_placement("rep", [alice, bob, carole])

    @edsl.computation
    def comp(x: edsl.Argument(alice, dtype=dtypes.float64)):
        with alice:
            xf = edsl.cast(x, dtype=dtypes.fixed(14, 23))
        with rep:
            y = edsl.sigmoid(edsl.mul(xf, xf))
        with bob:
            return edsl.cast(y, dtype=dtypes.float64)

    traced = trace(comp)
    data = utils.serialize_computation(traced)
    back = utils.deserialize_computation(data)
    assert set(back.operations) == set(traced.operations)
    for name, op in traced.operations.items():
        assert back.operation(name) == op
    from moose_amd.compiler.from_edsl import convert

    native = convert(back)
    kinds = {op.kind for op in native.operations}
    assert {"Input", "Cast", "Mul", "Sigmoid", "Output"} <= kinds
    mul = [op for op in native.operations if op.kind == "Mul"][0]
    assert mul.sig.ret.to_textual() == "Tensor<Fixed128(14, 23)>"
