"""Ring-level dialect programs on replicated and additive placements through the
declarative dispatch table (runtime/dispatch.py; reference kernel tables
moose/src/kernels/*.rs): textual computations mixing Share / ring arithmetic with public
operands / bit decomposition and composition / ShlDim / RepToAdt / AdtToRep / Reveal."""
import numpy as np
import pytest

from moose_amd.ir.computation import Computation
from moose_amd.runtime import dispatch
from moose_amd.runtime.local import LocalMooseRuntime

REP = "@Replicated(alice, bob, carole)"
M64 = (1 << 64) - 1


def run(body, ring=64, x=(5, 7, 2**63 + 11), y=(3, 2, 9)):
    R = f"Ring{ring}"
    src = f"""x = Constant{{value=Host{R}Tensor({list(x)})}}: () -> Host{R}Tensor @Host(alice)
y = Constant{{value=Host{R}Tensor({list(y)})}}: () -> Host{R}Tensor @Host(bob)
xs = Share: (Host{R}Tensor) -> Replicated{R}Tensor (x) {REP}
ys = Share: (Host{R}Tensor) -> Replicated{R}Tensor (y) {REP}
{body.replace("R_", R)}
"""
    rt = LocalMooseRuntime(["alice", "bob", "carole"], device="cpu")
    out = rt.evaluate_compiled(Computation.from_textual(src), {})["output_0"]
    return [int(v) for v in np.asarray(out, dtype=object).reshape(-1)]


def reveal(name, ty="Replicated{R}Tensor", host_ty="HostR_Tensor"):
    ty = ty.replace("{R}", "R_")
    return f"""out = Reveal: ({ty}) -> {host_ty} ({name}) @Host(alice)
output = Output{{tag = "output_0"}}: ({host_ty}) -> {host_ty} (out) @Host(alice)"""


X, Y = (5, 7, 2**63 + 11), (3, 2, 9)


@pytest.mark.parametrize("ring", [64, 128])
@pytest.mark.parametrize("op,f", [("Add", lambda a, b: a + b), ("Sub", lambda a, b: a - b),
                                  ("Mul", lambda a, b: a * b)])
def test_rep_ring_binops(ring, op, f):
    body = f"z = {op}: (ReplicatedR_Tensor, ReplicatedR_Tensor) -> ReplicatedR_Tensor (xs, ys) {REP}\n"
    got = run(body + reveal("z"), ring)
    assert got == [f(a, b) % (1 << ring) for a, b in zip(X, Y)]


@pytest.mark.parametrize("op,f", [("Add", lambda a, b: a + b), ("Sub", lambda a, b: a - b),
                                  ("Mul", lambda a, b: a * b)])
def test_rep_ring_with_public_operand(op, f):
    body = f"z = {op}: (ReplicatedR_Tensor, HostR_Tensor) -> ReplicatedR_Tensor (xs, y) {REP}\n"
    assert run(body + reveal("z")) == [f(a, b) & M64 for a, b in zip(X, Y)]
    body = f"z = {op}: (HostR_Tensor, ReplicatedR_Tensor) -> ReplicatedR_Tensor (y, xs) {REP}\n"
    assert run(body + reveal("z")) == [f(b, a) & M64 for a, b in zip(X, Y)]


def test_rep_unary_sum_addn_shl():
    body = f"""n = Neg: (ReplicatedR_Tensor) -> ReplicatedR_Tensor (xs) {REP}
s = AddN: [ReplicatedR_Tensor] -> ReplicatedR_Tensor (xs, ys, n) {REP}
h = Shl {{amount = 3}}: (ReplicatedR_Tensor) -> ReplicatedR_Tensor (s) {REP}
t = Sum {{axis = 0}}: (ReplicatedR_Tensor) -> ReplicatedR_Tensor (h) {REP}
"""
    assert run(body + reveal("t")) == [(sum(Y) << 3) & M64]


def test_rep_dot_ring_and_public():
    A = [[1, 2], [3, 4]]
    src = f"""a = Constant{{value=HostRing64Tensor({A})}}: () -> HostRing64Tensor @Host(alice)
b = Constant{{value=HostRing64Tensor([[5, 6], [7, 8]])}}: () -> HostRing64Tensor @Host(bob)
as_ = Share: (HostRing64Tensor) -> ReplicatedRing64Tensor (a) {REP}
bs = Share: (HostRing64Tensor) -> ReplicatedRing64Tensor (b) {REP}
d = Dot: (ReplicatedRing64Tensor, ReplicatedRing64Tensor) -> ReplicatedRing64Tensor (as_, bs) {REP}
e = Dot: (ReplicatedRing64Tensor, HostRing64Tensor) -> ReplicatedRing64Tensor (d, b) {REP}
out = Reveal: (ReplicatedRing64Tensor) -> HostRing64Tensor (e) @Host(alice)
output = Output{{tag = "output_0"}}: (HostRing64Tensor) -> HostRing64Tensor (out) @Host(alice)"""
    rt = LocalMooseRuntime(["alice", "bob", "carole"], device="cpu")
    got = np.asarray(rt.evaluate_compiled(Computation.from_textual(src), {})["output_0"])
    B = np.array([[5, 6], [7, 8]])
    np.testing.assert_array_equal(got.astype(np.int64), np.array(A) @ B @ B)


@pytest.mark.parametrize("ring", [64, 128])
def test_bit_decompose_compose_roundtrip(ring):
    body = f"""b = BitDecompose: (ReplicatedR_Tensor) -> ReplicatedBitArray{ring} (xs) {REP}
c = BitCompose: (ReplicatedBitArray{ring}) -> ReplicatedR_Tensor (b) {REP}
"""
    assert run(body + reveal("c"), ring) == [v % (1 << ring) for v in X]


def test_shl_dim_on_bit_array():
    body = f"""b = BitDecompose: (ReplicatedR_Tensor) -> ReplicatedBitArray64 (xs) {REP}
s = ShlDim {{amount = 5, bit_length = 64}}: (ReplicatedBitArray64) -> ReplicatedBitArray64 (b) {REP}
c = BitCompose: (ReplicatedBitArray64) -> ReplicatedR_Tensor (s) {REP}
"""
    assert run(body + reveal("c")) == [(v << 5) & M64 for v in X]


def test_msb_bit_and_ring_forms():
    body = f"m = Msb: (ReplicatedR_Tensor) -> ReplicatedR_Tensor (xs) {REP}\n"
    assert run(body + reveal("m")) == [v >> 63 for v in X]
    body = f"""b = BitDecompose: (ReplicatedR_Tensor) -> ReplicatedBitArray64 (xs) {REP}
e = BitExtract {{bit_idx = 63}}: (ReplicatedBitArray64) -> ReplicatedBitTensor (b) {REP}
r = RingInject {{bit_idx = 2}}: (ReplicatedBitTensor) -> ReplicatedR_Tensor (e) {REP}
"""
    assert run(body + reveal("r")) == [(v >> 63) << 2 for v in X]


def test_equal_mux_abs():
    body = f"""e = Equal: (ReplicatedR_Tensor, ReplicatedR_Tensor) -> ReplicatedR_Tensor (xs, ys) {REP}
m = Mux: (ReplicatedR_Tensor, ReplicatedR_Tensor, ReplicatedR_Tensor) -> ReplicatedR_Tensor (e, xs, ys) {REP}
"""
    assert run(body + reveal("m"), x=(4, 9, 1), y=(4, 2, 1)) == [4, 2, 1]
    body = f"a = Abs: (ReplicatedR_Tensor) -> ReplicatedR_Tensor (xs) {REP}\n"
    assert run(body + reveal("a"), x=(5, M64 - 6, 0)) == [5, 7, 0]


@pytest.mark.parametrize("ring", [64, 128])
def test_rep_to_adt_and_back(ring):
    body = f"""a = RepToAdt: (ReplicatedR_Tensor) -> AdditiveR_Tensor (xs) @Additive(alice, bob)
b = Add: (AdditiveR_Tensor, HostR_Tensor) -> AdditiveR_Tensor (a, y) @Additive(alice, bob)
c = AdtToRep: (AdditiveR_Tensor) -> ReplicatedR_Tensor (b) {REP}
"""
    assert run(body + reveal("c"), ring) == [(a + b) % (1 << ring) for a, b in zip(X, Y)]
    body2 = f"""a = RepToAdt: (ReplicatedR_Tensor) -> AdditiveR_Tensor (xs) @Additive(alice, bob)
n = Neg: (AdditiveR_Tensor) -> AdditiveR_Tensor (a) @Additive(alice, bob)
"""
    got = run(body2 + reveal("n", "AdditiveR_Tensor"), ring)
    assert got == [(-a) % (1 << ring) for a in X]


def test_table_covers_the_reference_dialect_ops():
    rep_ops = set(dispatch.ops_for("rep"))
    for op in ("Add", "Sub", "Mul", "Dot", "Neg", "Sum", "AddN", "Shl", "ShlDim", "TruncPr",
               "BitDecompose", "BitCompose", "BitExtract", "RingInject", "Msb", "Equal",
               "EqualZero", "Mux", "Xor", "And", "Or", "AdtToRep", "Share", "Abs", "Relu",
               "Concat", "Reshape", "ExpandDims", "Transpose", "Slice"):
        assert op in rep_ops, op
    assert {"RepToAdt", "Add", "Sub", "Mul", "Neg", "Shl"} <= set(dispatch.ops_for("adt"))
