"""Textual host computations executed end to end by both executors -- the port of the
reference's sync-vs-async execution matrix (moose/src/execution/mod.rs:133-957): every
case runs once on the program-order GraphExecutor ("sync", the reference's SyncSession)
and once on the native dataflow scheduler with worker threads ("async", AsyncSession).

Parity notes: DeriveSeed's concrete bytes (mod.rs:193-196) come from the reference's
seed derivation; ours derives seeds with its own PRF, so that case checks determinism and
non-zero output only ("parity unpinned")."""
import numpy as np
import pytest
import torch

from moose_amd.ir.computation import Computation
from moose_amd.runtime.dataflow import run_dataflow
from moose_amd.runtime.distributed import _host_numpy
from moose_amd.runtime.graph_executor import GraphExecutor

MODES = ["sync", "async"]


def run(src, mode, arguments=None, storage=None):
    comp = Computation.from_textual(src)
    storage = storage if storage is not None else {"alice": {}, "bob": {}}
    ex = GraphExecutor(torch.device("cpu"), storage)
    if mode == "sync":
        outs = ex.run(comp, dict(arguments or {}))
    else:
        outs = run_dataflow(ex, comp, dict(arguments or {}), workers=4)
    return {k: _host_numpy(v) for k, v in outs.items()}, storage


def out0(src, mode, **kw):
    return run(src, mode, **kw)[0]["output_0"]


@pytest.mark.parametrize("mode", MODES)
def test_eager_executor(mode):  # mod.rs:133-167
    body = "\n".join(
        f"x{i} = SampleSeeded{{}}: (HostShape, HostSeed) -> HostRing64Tensor (shape, seed) @Host(alice)"
        for i in range(100))
    src = f"""key = PrfKeyGen: () -> HostPrfKey () @Host(alice)
seed = DeriveSeed {{sync_key = [1, 2, 3]}}: (HostPrfKey) -> HostSeed (key) @Host(alice)
shape = Constant{{value = HostShape([2, 3])}}: () -> HostShape @Host(alice)
{body}
z = Output{{tag = "output_0"}}: (HostRing64Tensor) -> HostRing64Tensor (x0) @Host(alice)"""
    outs, _ = run(src, mode)
    assert list(outs) == ["output_0"]
    assert np.asarray(outs["output_0"]).shape == (2, 3)


@pytest.mark.parametrize("mode", MODES)
def test_constants_derive_seed(mode):  # mod.rs:169-199
    src = """key = Constant{value=HostPrfKey(00000000000000000000000000000000)}: () -> HostPrfKey @Host(alice)
seed = DeriveSeed {sync_key = [1, 2, 3]}: (HostPrfKey) -> HostSeed (key) @Host(alice)
output = Output{tag = "output_0"}: (HostSeed) -> HostSeed (seed) @Host(alice)"""
    def seed():
        v = out0(src, mode)
        return bytes(v) if isinstance(v, (bytes, bytearray)) else bytes(np.asarray(v, np.uint8))

    a, b = seed(), seed()
    assert len(a) == 16 and a != bytes(16)
    assert a == b  # a function of (key, sync_key)


@pytest.mark.parametrize("mode", MODES)
def test_constants_sample_ring(mode):  # mod.rs:201-222
    src = """seed = Constant{value=HostSeed(00000000000000000000000000000000)}: () -> HostSeed @Host(alice)
xshape = Constant{value=HostShape([2, 2])}: () -> HostShape @Host(alice)
sampled = SampleSeeded{}: (HostShape, HostSeed) -> HostRing64Tensor (xshape, seed) @Host(alice)
shape = Shape: (HostRing64Tensor) -> HostShape (sampled) @Host(alice)
output = Output{tag = "output_0"}: (HostShape) -> HostShape (shape) @Host(alice)"""
    assert tuple(out0(src, mode)) == (2, 2)


@pytest.mark.parametrize("mode", MODES)
def test_standard_input(mode):  # mod.rs:224-245
    src = """x = Input {arg_name = "x"}: () -> HostInt64Tensor @Host(alice)
y = Input {arg_name = "y"}: () -> HostInt64Tensor @Host(alice)
z = Add: (HostInt64Tensor, HostInt64Tensor) -> HostInt64Tensor (x, y) @Host(alice)
output = Output{tag = "output_0"}: (HostInt64Tensor) -> HostInt64Tensor (z) @Host(alice)"""
    got = out0(src, mode, arguments={"x": np.array([5], np.int64), "y": np.array([10], np.int64)})
    np.testing.assert_array_equal(got, [15])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("ty,arr", [("HostInt64Tensor", np.array([8], np.int64)),
                                    ("HostInt32Tensor", np.array([8], np.int32)),
                                    ("HostFloat32Tensor", np.array([8], np.float32)),
                                    ("HostFloat64Tensor", np.array([8], np.float64))])
def test_load_save(mode, ty, arr):  # mod.rs:247-311
    src = f"""x_uri = Input {{arg_name="x_uri"}}: () -> HostString () @Host(alice)
x_query = Input {{arg_name="x_query"}}: () -> HostString () @Host(alice)
saved_uri = Constant{{value = HostString("saved_data")}}: () -> HostString () @Host(alice)
x = Load: (HostString, HostString) -> {ty} (x_uri, x_query) @Host(alice)
save = Save: (HostString, {ty}) -> HostUnit (saved_uri, x) @Host(alice)
output = Output{{tag = "output_0"}}: (HostUnit) -> HostUnit (save) @Host(alice)"""
    storage = {"alice": {"input_data": arr}, "bob": {}}
    run(src, mode, arguments={"x_uri": "input_data", "x_query": ""}, storage=storage)
    saved = storage["alice"]["saved_data"]
    saved = saved.numpy() if isinstance(saved, torch.Tensor) else np.asarray(saved)
    np.testing.assert_array_equal(saved, arr)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("axis,want", [(0, [[1, 2], [3, 4], [5, 6], [7, 8]]),
                                       (1, [[1, 2, 5, 6], [3, 4, 7, 8]])])
def test_standard_concatenate(mode, axis, want):  # mod.rs:313-356
    src = f"""x_0 = Constant{{value=HostInt64Tensor([[1,2], [3,4]])}}: () -> HostInt64Tensor @Host(alice)
x_1 = Constant{{value=HostInt64Tensor([[5, 6], [7,8]])}}: () -> HostInt64Tensor @Host(alice)
concatenated = Concat {{axis={axis}}}: [HostInt64Tensor] -> HostInt64Tensor (x_0, x_1) @Host(alice)
output = Output{{tag = "output_0"}}: (HostInt64Tensor) -> HostInt64Tensor (concatenated) @Host(alice)"""
    np.testing.assert_array_equal(out0(src, mode), want)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("op,want", [("Add", 8), ("Sub", 2), ("Mul", 15), ("Div", 1)])
def test_standard_op(mode, op, want):  # mod.rs:358-397 (operands on two hosts)
    src = f"""x0 = Constant{{value=HostInt64Tensor([5])}}: () -> HostInt64Tensor @Host(alice)
x1 = Constant{{value=HostInt64Tensor([3])}}: () -> HostInt64Tensor @Host(bob)
res = {op}: (HostInt64Tensor, HostInt64Tensor) -> HostInt64Tensor (x0, x1) @Host(alice)
output = Output{{tag = "output_0"}}: (HostInt64Tensor) -> HostInt64Tensor (res) @Host(alice)"""
    np.testing.assert_array_equal(out0(src, mode), [want])


@pytest.mark.parametrize("mode", MODES)
def test_standard_dot(mode):  # mod.rs:399-430
    src = """x0 = Constant{value=HostFloat32Tensor([[1.0, 2.0], [3.0, 4.0]])}: () -> HostFloat32Tensor @Host(alice)
x1 = Constant{value=HostFloat32Tensor([[1.0, 0.0], [0.0, 1.0]])}: () -> HostFloat32Tensor @Host(bob)
res = Dot: (HostFloat32Tensor, HostFloat32Tensor) -> HostFloat32Tensor (x0, x1) @Host(alice)
output = Output{tag = "output_0"}: (HostFloat32Tensor) -> HostFloat32Tensor (res) @Host(alice)"""
    np.testing.assert_array_equal(out0(src, mode), [[1.0, 2.0], [3.0, 4.0]])


@pytest.mark.parametrize("mode", MODES)
def test_standard_inverse(mode):  # mod.rs:432-455
    src = """x = Constant{value=HostFloat32Tensor([[3.0, 2.0], [2.0, 3.0]])} : () -> HostFloat32Tensor @Host(alice)
x_inv = Inverse : (HostFloat32Tensor) -> HostFloat32Tensor (x) @Host(alice)
output = Output{tag = "output_0"}: (HostFloat32Tensor) -> HostFloat32Tensor (x_inv) @Host(alice)"""
    np.testing.assert_allclose(out0(src, mode), [[0.6, -0.4], [-0.4, 0.6]], rtol=1e-6)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("ty,np_dtype", [("HostFloat32Tensor", np.float32),
                                         ("HostFloat64Tensor", np.float64),
                                         ("HostInt64Tensor", np.int64)])
def test_standard_ones(mode, ty, np_dtype):  # mod.rs:457-516
    src = f"""s = Constant{{value=HostShape([2, 2])}}: () -> HostShape @Host(alice)
r = Ones : (HostShape) -> {ty} (s) @Host(alice)
output = Output{{tag = "output_0"}} : ({ty}) -> {ty} (r) @Host(alice)"""
    got = np.asarray(out0(src, mode))
    assert got.dtype == np_dtype
    np.testing.assert_array_equal(got, np.ones((2, 2)))


@pytest.mark.parametrize("mode", MODES)
def test_standard_shape(mode):  # mod.rs:518-538
    src = """x = Constant{value = HostFloat32Tensor([[1.0, 2.0], [3.0, 4.0]])}: () -> HostFloat32Tensor @Host(alice)
shape = Shape: (HostFloat32Tensor) -> HostShape (x) @Host(alice)
output = Output{tag = "output_0"}: (HostShape) -> HostShape (shape) @Host(alice)"""
    assert tuple(out0(src, mode)) == (2, 2)


@pytest.mark.parametrize("mode", MODES)
def test_shape_slice(mode):  # mod.rs:540-558
    src = """x = Constant{value = HostShape([2, 3, 4, 5])}: () -> HostShape @Host(alice)
slice = Slice {slice = {start = 1, end = 3}}: (HostShape) -> HostShape (x) @Host(alice)
output = Output{tag = "output_0"}: (HostShape) -> HostShape (slice) @Host(alice)"""
    assert tuple(out0(src, mode)) == (3, 4)


@pytest.mark.parametrize("mode", MODES)
def test_standard_expand_dims(mode):  # mod.rs:560-581
    src = """x = Constant{value = HostInt64Tensor([1, 2])}: () -> HostInt64Tensor @Host(alice)
expand_dims = ExpandDims {axis = [1]}: (HostInt64Tensor) -> HostInt64Tensor (x) @Host(alice)
output = Output{tag = "output_0"}: (HostInt64Tensor) -> HostInt64Tensor (expand_dims) @Host(alice)"""
    got = np.asarray(out0(src, mode))
    assert got.shape == (2, 1)
    np.testing.assert_array_equal(got.reshape(-1), [1, 2])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("op,axis,want", [("Sum", None, 10.0), ("Sum", 0, [4.0, 6.0]),
                                          ("Sum", 1, [3.0, 7.0]), ("Mean", None, 2.5),
                                          ("Mean", 0, [2.0, 3.0]), ("Mean", 1, [1.5, 3.5])])
def test_standard_reduce_op(mode, op, axis, want):  # mod.rs:583-684
    attrs = "{}" if axis is None else f"{{axis={axis}}}"
    src = f"""s = Constant{{value=HostFloat32Tensor([[1, 2], [3, 4]])}}: () -> HostFloat32Tensor @Host(alice)
r = {op} {attrs}: (HostFloat32Tensor) -> HostFloat32Tensor (s) @Host(alice)
output = Output{{tag = "output_0"}} : (HostFloat32Tensor) -> HostFloat32Tensor (r) @Host(alice)"""
    np.testing.assert_allclose(np.asarray(out0(src, mode)).reshape(np.shape(want)), want)


@pytest.mark.parametrize("mode", MODES)
def test_standard_transpose(mode):  # mod.rs:686-704
    src = """s = Constant{value=HostInt64Tensor([[1,2], [3, 4]])}: () -> HostInt64Tensor @Host(alice)
r = Transpose : (HostInt64Tensor) -> HostInt64Tensor (s) @Host(alice)
output = Output{tag = "output_0"} : (HostInt64Tensor) -> HostInt64Tensor (r) @Host(alice)"""
    np.testing.assert_array_equal(out0(src, mode), [[1, 3], [2, 4]])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("col,want", [(True, [[1.0], [1.0], [1.0]]), (False, [[1.0, 1.0, 1.0]])])
def test_standard_atleast_2d(mode, col, want):  # mod.rs:706-731
    src = f"""x = Constant{{value=HostFloat64Tensor([1.0, 1.0, 1.0])}}: () -> HostFloat64Tensor @Host(alice)
res = AtLeast2D {{ to_column_vector = {str(col).lower()} }} : (HostFloat64Tensor) -> HostFloat64Tensor (x) @Host(alice)
output = Output{{tag = "output_0"}} : (HostFloat64Tensor) -> HostFloat64Tensor (res) @Host(alice)"""
    np.testing.assert_array_equal(out0(src, mode), want)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("op,want", [("Add", 5), ("Mul", 6), ("Sub", 1)])
def test_ring_binop_invocation(mode, op, want):  # mod.rs:733-762
    src = f"""x =  Constant{{value=HostRing64Tensor([3])}}: () -> HostRing64Tensor @Host(alice)
y = Constant{{value=HostRing64Tensor([2])}}: () -> HostRing64Tensor @Host(alice)
res = {op} : (HostRing64Tensor, HostRing64Tensor) -> HostRing64Tensor (x, y) @Host(alice)
output = Output{{tag = "output_0"}} : (HostRing64Tensor) -> HostRing64Tensor (res) @Host(alice)"""
    np.testing.assert_array_equal(np.asarray(out0(src, mode)).astype(np.uint64), [want])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("x,y,want", [("[[1, 2], [3, 4]]", "[[1, 0], [0, 1]]", [[1, 2], [3, 4]]),
                                      ("[[1, 2], [3, 4]]", "[1, 1]", [3, 7]),
                                      ("[1, 1]", "[[1, 2], [3, 4]]", [4, 6])])
def test_ring_dot_invocation(mode, x, y, want):  # mod.rs:764-841
    src = f"""x = Constant{{value=HostRing64Tensor({x})}}: () -> HostRing64Tensor @Host(alice)
y = Constant{{value=HostRing64Tensor({y})}}: () -> HostRing64Tensor @Host(alice)
res = Dot : (HostRing64Tensor, HostRing64Tensor) -> HostRing64Tensor (x, y) @Host(alice)
output = Output{{tag = "output_0"}} : (HostRing64Tensor) -> HostRing64Tensor (res) @Host(alice)"""
    np.testing.assert_array_equal(np.asarray(out0(src, mode)).astype(np.uint64), want)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("ring,shape,want", [("Ring64", "2", [1, 1]), ("Ring128", "2", [1, 1]),
                                             ("Ring64", "2, 1", [[1], [1]]),
                                             ("Ring64", "2, 2", [[1, 1], [1, 1]]),
                                             ("Ring64", "1, 2", [[1, 1]]),
                                             ("Ring128", "2, 3", [[1, 1, 1], [1, 1, 1]])])
def test_fill(mode, ring, shape, want):  # mod.rs:843-906
    src = f"""shape = Constant{{value=HostShape([{shape}])}}: () -> HostShape @Host(alice)
res = Fill {{value = {ring}(1)}} : (HostShape) -> Host{ring}Tensor (shape) @Host(alice)
output = Output{{tag = "output_0"}} : (Host{ring}Tensor) -> Host{ring}Tensor (res) @Host(alice)"""
    got = np.asarray(out0(src, mode))
    np.testing.assert_array_equal(np.vectorize(int, otypes=[object])(got), want)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("ty", ["HostRing64Tensor", "HostRing128Tensor"])
def test_ring_bitwise_ops(mode, ty):  # mod.rs:908-957
    src = f"""x = Constant{{value={ty}([4, 4])}}: () -> {ty} @Host(alice)
res = Shr {{amount = 1}}: ({ty}) -> {ty} (x) @Host(alice)
output = Output{{tag = "output_0"}}: ({ty}) -> {ty} (res) @Host(alice)"""
    got = np.asarray(out0(src, mode))
    np.testing.assert_array_equal(np.vectorize(int, otypes=[object])(got), [2, 2])
