"""Bincode-style binary computation format (reference computation.rs:1837-1844,
``elk compile -f bincode``): exact round trips of every textual fixture, including the
reference's 19k-op lowered benchmark graph, and the elk CLI path."""
import glob
import os

import numpy as np
import pytest

from moose_amd.cli import elk
from moose_amd.ir.bincode import BincodeError
from moose_amd.ir.computation import Computation

REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = (sorted(glob.glob(os.path.join(REPO, "examples", "*.moose")))
         + sorted(glob.glob(os.path.join(REF, "tutorials", "*.moose")))
         + sorted(glob.glob(os.path.join(REF, "moose", "benches", "*.moose"))))


@pytest.mark.parametrize("path", FILES)
def test_round_trip_is_exact(path):
    comp = Computation.from_textual(open(path).read())
    data = comp.to_bincode()
    back = Computation.from_bincode(data)
    assert back.to_textual() == comp.to_textual()
    assert back.to_bincode() == data


def test_constants_and_attributes():
    src = (
        'a = Constant{value = HostRing128Tensor([[340282366920938463463374607431768211455, 1]])}: '
        '() -> HostRing128Tensor () @Host(alice)\n'
        'b = Constant{value = HostFloat32Tensor([1.5, -2.0])}: () -> HostFloat32Tensor () @Host(alice)\n'
        'c = Slice{slice = {start = 1, end = 3}}: (HostFloat32Tensor) -> HostFloat32Tensor (b) @Host(alice)\n'
        's = Send{rendezvous_key = 0102, receiver = "bob"}: (HostFloat32Tensor) -> HostUnit (c) @Host(alice)\n'
        'r = Receive{rendezvous_key = 0102, sender = "alice"}: () -> HostFloat32Tensor () @Host(bob)\n')
    comp = Computation.from_textual(src)
    back = Computation.from_bincode(comp.to_bincode())
    assert back.operations[0].attrs["value"].value[0, 0] == (1 << 128) - 1
    np.testing.assert_array_equal(back.operations[1].attrs["value"].value, [1.5, -2.0])
    assert back.operations[1].attrs["value"].value.dtype == np.float32
    assert back.to_textual() == comp.to_textual()


def test_corrupt_payloads_are_rejected():
    comp = Computation.from_textual(
        'x = Constant{value = Float64(1.0)}: () -> Float64 () @Host(a)\n')
    data = comp.to_bincode()
    with pytest.raises(BincodeError):
        Computation.from_bincode(data[:-3])
    with pytest.raises(BincodeError):
        Computation.from_bincode(b"XXXX" + data[4:])
    with pytest.raises(BincodeError):
        Computation.from_bincode(data + b"\x00")


def test_elk_compile_to_and_from_bincode(tmp_path):
    src = os.path.join(REPO, "examples", "dot.moose")
    out = tmp_path / "dot.bin"
    assert elk.main(["compile", src, "-o", str(out), "-f", "bincode", "-p", "typing"]) == 0
    again = tmp_path / "dot.moose"
    assert elk.main(["compile", str(out), "-i", "bincode", "-o", str(again), "-p", ""]) == 0
    assert Computation.from_textual(open(again).read()).to_textual() == \
        Computation.from_bincode(open(out, "rb").read()).to_textual()
