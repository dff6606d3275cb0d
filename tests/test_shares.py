"""Pre-shared replicated inputs and per-party share checkpoints.

Reference parity: ``moose/src/replicated/input.rs`` (``"{arg}/{role}/share{i}"``
arguments, Fixed64 -> (14,23), Fixed128 -> (24,40)) and its tests
(``input.rs:121-211``: inputs assembled from per-role shares reveal to the secret).
The checkpoint half is new: Save/Load on a replicated placement keep each
party's shares in its own storage only."""
import numpy as np
import pytest
import torch

import moose_amd as pm
from moose_amd.ir.computation import Computation
from moose_amd.runtime.distributed import DistributedMooseRuntime
from moose_amd.runtime.local import LocalMooseRuntime
from moose_amd.utils import checkpoint

ROLES = ["alice", "bob", "carole"]
M128 = 1 << 128


def _split(values, bits, rng):
    """Three additive shares of python ints mod 2^bits."""
    mod = 1 << bits
    a = [int.from_bytes(rng.bytes(bits // 8), "little") for _ in values]
    b = [int.from_bytes(rng.bytes(bits // 8), "little") for _ in values]
    c = [(v - x - y) % mod for v, x, y in zip(values, a, b)]
    return [a, b, c]


def _enc(vals, bits, shape):
    if bits == 64:
        return np.array(vals, dtype=np.uint64).reshape(shape)
    return np.array([[v & (2**64 - 1), v >> 64] for v in vals], dtype=np.uint64).reshape(
        shape + (2,))


def _preshared_args(name, x, bits, frac, seed=0):
    rng = np.random.default_rng(seed)
    enc = [int(round(v * 2**frac)) % (1 << bits) for v in x.reshape(-1)]
    sh = _split(enc, bits, rng)
    args = {}
    for i, r in enumerate(ROLES):
        args[f"{name}/{r}/share{i}"] = _enc(sh[i], bits, x.shape)
        args[f"{name}/{r}/share{(i + 1) % 3}"] = _enc(sh[(i + 1) % 3], bits, x.shape)
    return args


def _placements():
    alice, bob, carole = (pm.host_placement(n) for n in ROLES)
    return alice, bob, carole, pm.replicated_placement("rep", players=[alice, bob, carole])


def _mul_and_save(fx):
    alice, bob, carole, rep = _placements()

    @pm.computation
    def f(x: pm.Argument(placement=rep, vtype=pm.TensorType(fx)),
          y: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            yf = pm.cast(y, dtype=fx)
        with rep:
            z = pm.mul(x, yf)
            s = pm.save("ckpt", z)
        with carole:
            out = pm.cast(z, dtype=pm.float64)
        return out, s

    return f


def _load_double(fx):
    alice, bob, carole, rep = _placements()

    @pm.computation
    def g():
        with rep:
            w = pm.load("ckpt", vtype=pm.TensorType(fx))
            w2 = pm.add(w, w)
        with carole:
            out = pm.cast(w2, dtype=pm.float64)
        return out

    return g


@pytest.mark.parametrize("bits,fx", [(128, pm.fixed(24, 40)), (64, pm.fixed(14, 23))])
def test_preshared_input_and_checkpoint_roundtrip(bits, fx, tmp_path):
    rng = np.random.default_rng(1)
    x, y = rng.uniform(-3, 3, (4, 5)), rng.uniform(-3, 3, (4, 5))
    args = dict(_preshared_args("x", x, bits, fx.fractional_precision), y=y)
    rt = LocalMooseRuntime(ROLES, device="cpu", fixedpoint_ring=bits)
    out = rt.evaluate_computation(_mul_and_save(fx), args)
    np.testing.assert_allclose(out["output_0"], x * y, atol=1e-5)
    # every party holds exactly its own pair (x_i, x_{i+1}) and the meta record
    for i, r in enumerate(ROLES):
        keys = {k for k in rt.storage[r] if k.startswith("ckpt/")}
        assert keys == {f"ckpt/{r}/share{i}", f"ckpt/{r}/share{(i + 1) % 3}", f"ckpt/{r}/meta"}
    # replicated consistency: the copies of x_i held by two parties agree
    for i in range(3):
        a = rt.storage[ROLES[i]][f"ckpt/{ROLES[i]}/share{i}"]
        b = rt.storage[ROLES[(i - 1) % 3]][f"ckpt/{ROLES[(i - 1) % 3]}/share{i}"]
        np.testing.assert_array_equal(a, b)
    # to disk and back into a fresh runtime; resume from the checkpoint
    assert checkpoint.save_all(rt.storage, str(tmp_path), prefixes=["ckpt"]) == 9
    restored = checkpoint.load_all(str(tmp_path))
    rt2 = LocalMooseRuntime(ROLES, device="cpu", fixedpoint_ring=bits,
                            storage_mapping=restored)
    out2 = rt2.evaluate_computation(_load_double(fx), {})
    np.testing.assert_allclose(out2["output_0"], 2 * x * y, atol=1e-5)


def test_preshared_ring_input_textual():
    """Reference-style textual computation: a ReplicatedRing64Tensor input revealed."""
    src = """
x = Input {arg_name = "x"}: () -> ReplicatedRing64Tensor @Replicated(alice, bob, carole)
y = Reveal: (ReplicatedRing64Tensor) -> HostRing64Tensor (x) @Host(carole)
output = Output{tag = "output"}: (HostRing64Tensor) -> HostRing64Tensor (y) @Host(carole)
"""
    comp = Computation.from_textual(src)
    vals = [1, 2, 3, 2**63 + 5]
    rng = np.random.default_rng(2)
    sh = _split(vals, 64, rng)
    args = {}
    for i, r in enumerate(ROLES):
        args[f"x/{r}/share{i}"] = np.array(sh[i], dtype=np.uint64)
        args[f"x/{r}/share{(i + 1) % 3}"] = np.array(sh[(i + 1) % 3], dtype=np.uint64)
    out = LocalMooseRuntime(ROLES, device="cpu").evaluate_computation(comp, args)
    got = [int(v) % 2**64 for v in np.asarray(out["output"]).reshape(-1)]
    assert got == vals


def test_missing_share_argument_is_an_error():
    fx = pm.fixed(24, 40)
    args = _preshared_args("x", np.ones((2, 2)), 128, 40)
    del args["x/bob/share2"]
    args["y"] = np.ones((2, 2))
    with pytest.raises(Exception, match="share2"):
        LocalMooseRuntime(ROLES, device="cpu").evaluate_computation(_mul_and_save(fx), args)


def test_distributed_checkpoint_stays_with_its_owner():
    """One process per party (gloo): each worker's storage receives only its own shares,
    and a second session resumes from them."""
    fx = pm.fixed(24, 40)
    rng = np.random.default_rng(4)
    x, y = rng.uniform(-2, 2, (3, 3)), rng.uniform(-2, 2, (3, 3))
    args = dict(_preshared_args("x", x, 128, 40, seed=5), y=y)
    rt = DistributedMooseRuntime(ROLES, backend="gloo", seed=2, timeout=300)
    out = rt.evaluate_computation(_mul_and_save(fx), args)
    np.testing.assert_allclose(np.asarray(out["output_0"], dtype=np.float64), x * y, atol=1e-5)
    for i, r in enumerate(ROLES):
        keys = {k for k in rt.storage[r] if k.startswith("ckpt/")}
        assert keys == {f"ckpt/{r}/share{i}", f"ckpt/{r}/share{(i + 1) % 3}", f"ckpt/{r}/meta"}
    out2 = rt.evaluate_computation(_load_double(fx), {})
    np.testing.assert_allclose(np.asarray(out2["output_0"], dtype=np.float64), 2 * x * y,
                               atol=1e-5)


@pytest.mark.gpu
def test_checkpoint_roundtrip_on_gpu():
    fx = pm.fixed(24, 40)
    rng = np.random.default_rng(6)
    x, y = rng.uniform(-3, 3, (64, 32)), rng.uniform(-3, 3, (64, 32))
    args = dict(_preshared_args("x", x, 128, 40), y=y)
    rt = LocalMooseRuntime(ROLES, device="cuda:0")
    out = rt.evaluate_computation(_mul_and_save(fx), args)
    np.testing.assert_allclose(out["output_0"], x * y, atol=1e-5)
    out2 = rt.evaluate_computation(_load_double(fx), {})
    np.testing.assert_allclose(out2["output_0"], 2 * x * y, atol=1e-5)
    assert torch.cuda.is_available()


def test_dialect_level_textual_computation():
    """Replicated dialect ops written directly in the textual format (as in the
    reference's execution tests): Share, TruncPr, Msb, Reveal, plus host ring ops."""
    plc = "@Replicated(alice, bob, carole)"
    src = f"""
x = Constant{{value = HostRing64Tensor([800, 1600, 18446744073709551416])}}: () -> HostRing64Tensor @Host(alice)
xs = Share: (HostRing64Tensor) -> ReplicatedRing64Tensor (x) {plc}
t = TruncPr{{amount = 2}}: (ReplicatedRing64Tensor) -> ReplicatedRing64Tensor (xs) {plc}
m = Msb: (ReplicatedRing64Tensor) -> ReplicatedBitTensor (xs) {plc}
tr = Reveal: (ReplicatedRing64Tensor) -> HostRing64Tensor (t) @Host(carole)
mr = Reveal: (ReplicatedBitTensor) -> HostBitTensor (m) @Host(carole)
sh = Shl{{amount = 3}}: (HostRing64Tensor) -> HostRing64Tensor (tr) @Host(carole)
o1 = Output{{tag = "t"}}: (HostRing64Tensor) -> HostRing64Tensor (sh) @Host(carole)
o2 = Output{{tag = "m"}}: (HostBitTensor) -> HostBitTensor (mr) @Host(carole)
"""
    comp = Computation.from_textual(src)
    out = LocalMooseRuntime(ROLES, device="cpu").evaluate_computation(comp, {})
    t = [int(v) % 2**64 for v in np.asarray(out["t"]).reshape(-1)]
    t = [v - 2**64 if v >= 2**63 else v for v in t]
    want = [200 * 8, 400 * 8, -50 * 8]
    assert all(abs(a - b) <= 8 for a, b in zip(t, want)), t
    assert [int(v) for v in np.asarray(out["m"]).reshape(-1)] == [0, 0, 1]


def test_dialect_equal_pow2_mirror_encode():
    """More dialect-level operators reachable from textual computations: Equal / Index on
    replicated rings, Pow2 on a replicated fixed-point tensor, Mirror/Demirror, and
    FixedpointEncode/Decode on a host."""
    plc = "@Replicated(alice, bob, carole)"
    src = f"""
a = Constant{{value = HostRing64Tensor([5, 7, 9])}}: () -> HostRing64Tensor @Host(alice)
b = Constant{{value = HostRing64Tensor([5, 8, 9])}}: () -> HostRing64Tensor @Host(bob)
ra = Share: (HostRing64Tensor) -> ReplicatedRing64Tensor (a) {plc}
rb = Share: (HostRing64Tensor) -> ReplicatedRing64Tensor (b) {plc}
eq = Equal: (ReplicatedRing64Tensor, ReplicatedRing64Tensor) -> ReplicatedBitTensor (ra, rb) {plc}
eqo = Reveal: (ReplicatedBitTensor) -> HostBitTensor (eq) @Host(carole)
x = Constant{{value = HostFloat64Tensor([0.5, -1.25, 2.0])}}: () -> HostFloat64Tensor @Host(alice)
xf = FixedpointEncode{{fractional_precision = 23, integral_precision = 14}}: (HostFloat64Tensor) -> HostFixed128Tensor (x) @Host(alice)
p = Pow2: (Tensor<Fixed128(14, 23)>) -> Tensor<Fixed128(14, 23)> (xf) {plc}
po = FixedpointDecode{{fractional_precision = 23}}: (HostFixed128Tensor) -> HostFloat64Tensor (p) @Host(carole)
m = Mirror: (HostFloat64Tensor) -> Mirrored3Float64 (x) @Mirrored3(alice, bob, carole)
md = Demirror: (Mirrored3Float64) -> HostFloat64Tensor (m) @Host(bob)
o1 = Output{{tag = "eq"}}: (HostBitTensor) -> HostBitTensor (eqo) @Host(carole)
o2 = Output{{tag = "pow2"}}: (HostFloat64Tensor) -> HostFloat64Tensor (po) @Host(carole)
o3 = Output{{tag = "mir"}}: (HostFloat64Tensor) -> HostFloat64Tensor (md) @Host(bob)
"""
    comp = Computation.from_textual(src)
    out = LocalMooseRuntime(ROLES, device="cpu").evaluate_computation(comp, {})
    assert [int(v) for v in np.asarray(out["eq"]).reshape(-1)] == [1, 0, 1]
    np.testing.assert_allclose(np.asarray(out["pow2"], dtype=np.float64),
                               2.0 ** np.array([0.5, -1.25, 2.0]), atol=1e-3)
    np.testing.assert_allclose(np.asarray(out["mir"], dtype=np.float64), [0.5, -1.25, 2.0])
