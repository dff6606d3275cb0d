"""Textual format: parse/print round trips (reference textual/parsing.rs tests and
computation.rs:1974-2009)."""
import glob

import numpy as np
import pytest

from moose_amd.ir import types as T
from moose_amd.ir.computation import Computation
from moose_amd.ir.computation import HostPlacement
from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ir.textual import ParseError
from moose_amd.ir.textual import parse_computation

REF_FILES = sorted(glob.glob("/root/reference/**/*.moose", recursive=True))


@pytest.mark.parametrize("path", REF_FILES, ids=lambda p: p.split("/reference/")[-1])
def test_reference_files_roundtrip(path):
    src = open(path).read()
    comp = parse_computation(src)
    assert len(comp) > 0
    txt = comp.to_textual()
    again = parse_computation(txt)
    assert again.to_textual() == txt
    comp.toposorted()  # send->receive edges resolve, no cycles


def test_dotprod_structure():
    comp = parse_computation(open("/root/reference/tutorials/dotprod.moose").read())
    kinds = [op.kind for op in comp]
    assert kinds == ["Constant", "Cast", "Constant", "Cast", "Dot", "Cast", "Output"]
    dot = comp.operations[4]
    assert dot.placement == ReplicatedPlacement(("player0", "player1", "player2"))
    assert dot.sig.ret == T.tensor(T.fixed128(24, 40))
    c = comp.operations[0].attrs["value"]
    np.testing.assert_array_equal(c.value, np.array([[1.0, 2.0, 3.0]]))


@pytest.mark.parametrize(
    "line",
    [
        'x = Constant{value = HostFloat32Tensor([1.0, 2.0])}: () -> HostFloat32Tensor () @Host(alice)',
        'x = Constant{value = HostShape([2, 3])}: () -> HostShape () @Host(alice)',
        'x = Constant{value = HostString("hello")}: () -> HostString () @Host(alice)',
        'x = Constant{value = Ring64(5)}: () -> Ring64 () @Host(alice)',
        "s = Send{rendezvous_key = 01000000000000000000000000000000, receiver = \"bob\"}: (HostFloat32Tensor) -> HostUnit (x) @Host(alice)",
        "r = Receive{rendezvous_key = 01000000000000000000000000000000, sender = \"alice\"}: () -> HostFloat32Tensor () @Host(bob)",
        "y = Sum{axis = 0}: (HostFloat32Tensor) -> HostFloat32Tensor (x) @Host(alice)",
        "y = Sum{}: (HostFloat32Tensor) -> HostFloat32Tensor (x) @Host(alice)",
        "y = ExpandDims{axis = [0, 2]}: (HostFloat32Tensor) -> HostFloat32Tensor (x) @Host(alice)",
        "y = Slice{slice = {start = 1, end = 3}}: (HostShape) -> HostShape (x) @Host(alice)",
        "y = RingFixedpointEncode{scaling_base = 2, scaling_exp = 40}: (HostFloat64Tensor) -> HostRing128Tensor (x) @Host(alice)",
        "y = Fill{value = Ring128(1)}: (HostShape) -> HostRing128Tensor (x) @Host(alice)",
        "y = ShlDim{amount = 1, bit_length = 128}: (HostBitTensor) -> HostBitTensor (x) @Host(alice)",
        "z = AddN: [Tensor<Fixed64(14, 23)>] -> Tensor<Fixed64(14, 23)> (a, b, c) @Replicated(alice, bob, carole)",
        "z = Dot: (Tensor<Float64>, Tensor<Float64>) -> Tensor<Float64> (a, b) @Mirrored3(alice, bob, carole)",
    ],
)
def test_line_roundtrip(line):
    comp = parse_computation(line)
    assert comp.to_textual() == line


def test_deprecated_aliases_and_comments():
    src = """
    // a comment
    k = PrimPrfKeyGen: () -> PrfKey () @Host(alice)
    s = PrimDeriveSeed{sync_key = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16]}: (PrfKey) -> Seed (k) @Host(alice)
    """
    comp = parse_computation(src)
    assert [op.kind for op in comp] == ["PrfKeyGen", "DeriveSeed"]
    assert comp.operations[1].attrs["sync_key"] == bytes(range(1, 17))
    assert comp.operations[0].sig.ret == T.HOST_PRF_KEY


def test_parse_errors_are_reported():
    with pytest.raises(ParseError):
        parse_computation("x = NotAnOp: () -> HostUnit () @Host(alice)")
    with pytest.raises(ParseError):
        parse_computation("x = Add: (HostFloat32Tensor) -> HostFloat32Tensor (a) @Replicated(a, b)")


def test_msgpack_roundtrip(tmp_path):
    comp = parse_computation(open("/root/reference/tutorials/dotprod-networked.moose").read())
    data = comp.to_msgpack()
    back = Computation.from_msgpack(data)
    assert back.to_textual() == comp.to_textual()
    p = tmp_path / "c.bin"
    comp.to_disk(p)
    assert Computation.from_disk(p).to_textual() == comp.to_textual()


def test_toposort_detects_cycles():
    comp = parse_computation(
        "a = Add: (HostFloat32Tensor, HostFloat32Tensor) -> HostFloat32Tensor (b, b) @Host(x)\n"
        "b = Add: (HostFloat32Tensor, HostFloat32Tensor) -> HostFloat32Tensor (a, a) @Host(x)"
    )
    with pytest.raises(ValueError):
        comp.toposorted()


def test_placement_kinds():
    comp = parse_computation("x = Identity: (HostFloat32Tensor) -> HostFloat32Tensor (y) @Host(alice)")
    assert comp.operations[0].placement == HostPlacement("alice")
