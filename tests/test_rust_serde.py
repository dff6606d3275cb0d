"""Rust-layout binary computations (reference ``NamedComputation::{to,from}_bincode`` and
``{to,from}_msgpack``, computation.rs:1797-1874).

Parity unpinned: the reference ships no binary fixtures.  The tests pin (a) exact round
trips of every textual fixture through both encodings, and (b) hand-assembled byte strings
of small computations, written out from the serde rules (bincode 1.3 default options;
rmp-serde 1.1 ``to_vec``) and the reference's type declarations, independently of the
encoder."""
import glob
import os
import struct

import numpy as np
import pytest

from moose_amd.cli import elk
from moose_amd.ir import rust_serde as RS
from moose_amd.ir.computation import Computation

REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = (sorted(glob.glob(os.path.join(REPO, "examples", "*.moose")))
         + sorted(glob.glob(os.path.join(REF, "tutorials", "*.moose")))
         + sorted(glob.glob(os.path.join(REF, "moose", "benches", "*.moose"))))
ENC = {"bincode": (RS.to_rust_bincode, RS.from_rust_bincode),
       "msgpack": (RS.to_rust_msgpack, RS.from_rust_msgpack)}


def _rust_ops(comp):
    return all(op.kind in RS.OPERATOR_VARIANTS for op in comp.operations)


@pytest.mark.parametrize("fmt", sorted(ENC))
@pytest.mark.parametrize("path", FILES, ids=os.path.basename)
def test_fixture_round_trip(path, fmt):
    comp = Computation.from_textual(open(path).read())
    assert _rust_ops(comp)
    enc, dec = ENC[fmt]
    data = enc(comp)
    back = dec(data)
    assert back.to_textual() == comp.to_textual()
    assert enc(back) == data


def test_variant_tables_follow_the_reference_declarations():
    assert len(RS.OPERATOR_VARIANTS) == 81
    assert RS.OPERATOR_VARIANTS[:3] == ["Abs", "Add", "And"]
    assert RS.OPERATOR_VARIANTS[-2:] == ["Demirror", "Mirror"]
    assert RS.TY_VARIANTS[0] == "Unknown" and RS.TY_VARIANTS[-1] == "Fixed"
    assert len(RS.TY_VARIANTS) == 66
    assert RS.CONSTANT_VARIANTS.index("Fixed") == 22


def _u32(v):
    return struct.pack("<I", v)


def _u64(v):
    return struct.pack("<Q", v)


def _s(x):
    b = x.encode()
    return _u64(len(b)) + b


def test_bincode_bytes_of_an_input_op():
    """x = Input{arg_name = "x"}: () -> HostFloat64Tensor () @Host(alice), by hand:
    operations: u64 1; name "x"; Operator::Input = variant 18; sig Nullary = 0 with
    ret Ty::HostFloat64Tensor = 18; arg_name "x"; inputs []; Placement::Host = 0, "alice"."""
    comp = Computation.from_textual(
        'x = Input{arg_name = "x"}: () -> HostFloat64Tensor () @Host(alice)\n')
    want = (_u64(1) + _s("x") + _u32(18) + _u32(0) + _u32(18) + _s("x") + _u64(0)
            + _u32(0) + _s("alice"))
    assert RS.to_rust_bincode(comp) == want
    assert RS.from_rust_bincode(want).to_textual() == comp.to_textual()


def test_bincode_bytes_of_attributes_and_constants():
    """Sum{axis = 0} (Option<usize>: tag 1 + u64), TruncPr (u32), a Fixed128 tensor type
    (Ty::Tensor = 7 with TensorDType::Fixed128 = 1 {i: u32, f: u32}), a replicated
    placement ([Role; 3] without a length), and a HostFloat64Tensor constant (ndarray
    {v = 1, dim, data} + its HostPlacement "TODO")."""
    comp = Computation.from_textual(
        'c = Constant{value = HostFloat64Tensor([[1.5, 2.0]])}: () -> HostFloat64Tensor () @Host(a)\n'
        's = Sum{axis = 0}: (HostFloat64Tensor) -> HostFloat64Tensor (c) @Host(a)\n'
        't = TruncPr{amount = 7}: (Tensor<Fixed128(24, 40)>) -> Tensor<Fixed128(24, 40)> (s) '
        '@Replicated(a, b, c)\n')
    host_a = _u32(0) + _s("a")
    op_c = (_s("c") + _u32(8) + _u32(0) + _u32(18)            # Constant, Nullary -> HostFloat64
            + _u32(8)                                          # Constant::HostFloat64Tensor
            + bytes([1]) + _u64(2) + _u64(1) + _u64(2)         # v, dim [1, 2]
            + _u64(2) + struct.pack("<dd", 1.5, 2.0)           # data
            + _s("TODO")                                       # constant's HostPlacement
            + _u64(0) + host_a)
    op_s = (_s("s") + _u32(47) + _u32(1) + _u32(18) + _u32(18)  # Sum, Unary
            + bytes([1]) + _u64(0)                               # Some(0usize)
            + _u64(1) + _s("c") + host_a)
    fx = _u32(7) + _u32(1) + _u32(24) + _u32(40)                 # Tensor<Fixed128(24, 40)>
    op_t = (_s("t") + _u32(78) + _u32(1) + fx + fx + _u32(7)     # TruncPr, amount: u32
            + _u64(1) + _s("s") + _u32(1) + _s("a") + _s("b") + _s("c"))
    want = _u64(3) + op_c + op_s + op_t
    assert RS.to_rust_bincode(comp) == want
    back = RS.from_rust_bincode(want)
    assert back.to_textual() == comp.to_textual()
    assert back.operations[0].attrs["value"].value.dtype == np.float64


def test_msgpack_bytes_of_an_input_op():
    """rmp-serde 1.1: structs as arrays, enum variants by name (newtype variant = one-entry
    map, unit variant = string)."""
    comp = Computation.from_textual(
        'x = Input{arg_name = "x"}: () -> HostFloat64Tensor () @Host(alice)\n')
    want = (b"\x91" + b"\x91"                                   # NamedComputation, Vec len 1
            + b"\x94" + b"\xa1x"                                 # Operation [name, ...]
            + b"\x81\xa5Input" + b"\x92"                         # {Input: [sig, arg_name]}
            + b"\x81\xa7Nullary" + b"\x91\xb1HostFloat64Tensor"  # {Nullary: [ret]}
            + b"\xa1x"                                           # arg_name
            + b"\x90"                                            # inputs []
            + b"\x81\xa4Host" + b"\x91\xa5alice")                # {Host: [owner]}
    assert RS.to_rust_msgpack(comp) == want
    assert RS.from_rust_msgpack(want).to_textual() == comp.to_textual()


def test_msgpack_u128_options_and_keys():
    comp = Computation.from_textual(
        'k = Constant{value = Ring128(340282366920938463463374607431768211455)}: () -> Ring128 () @Host(a)\n'
        'm = Mean{axis = None}: (HostFloat64Tensor) -> HostFloat64Tensor (k) @Host(a)\n'
        's = Send{rendezvous_key = 0102, receiver = "b"}: (HostFloat64Tensor) -> HostUnit (m) @Host(a)\n')
    data = RS.to_rust_msgpack(comp)
    assert b"\x81\xa7Ring128\xc4\x10" + b"\xff" * 16 in data       # u128 = 16-byte bin
    assert b"\x81\xa4Mean\x92" in data and b"\xc0\x91\xa1k" in data  # None = nil
    key = bytes(14) + b"\x01\x02"
    assert b"\xdc\x00\x10" + key + b"\xa1b" in data                 # [u8; 16]: array of 16
    assert RS.from_rust_msgpack(data).to_textual() == comp.to_textual()


def test_constants_of_every_kind_round_trip():
    src = (
        'a = Constant{value = HostRing128Tensor([[340282366920938463463374607431768211455, 1]])}: '
        '() -> HostRing128Tensor () @Host(alice)\n'
        'b = Constant{value = HostFloat32Tensor([1.5, -2.0])}: () -> HostFloat32Tensor () @Host(alice)\n'
        'c = Constant{value = HostInt16Tensor([-3, 4])}: () -> HostInt16Tensor () @Host(alice)\n'
        'd = Constant{value = HostBitTensor([[1, 0, 1], [1, 1, 0]])}: () -> HostBitTensor () @Host(alice)\n'
        'e = Constant{value = HostShape([2, 3])}: () -> HostShape () @Host(alice)\n'
        'f = Constant{value = HostString("hi")}: () -> HostString () @Host(alice)\n'
        'g = Constant{value = Float32(0.5)}: () -> Float32 () @Host(alice)\n'
        'h = Constant{value = Ring64(18446744073709551615)}: () -> Ring64 () @Host(alice)\n'
        'i = Slice{slice = [{start = 1, end = 3}, {start = -2, step = 2}]}: '
        '(HostFloat32Tensor) -> HostFloat32Tensor (b) @Host(alice)\n'
        'j = ExpandDims{axis = [0, 2]}: (HostFloat32Tensor) -> HostFloat32Tensor (i) @Host(alice)\n'
        'k = AddN: [ReplicatedRing64Tensor] -> ReplicatedRing64Tensor (h, h) @Replicated(alice, bob, carole)\n'
        'l = Identity: (Shape<Replicated>) -> Shape<Replicated> (e) @Additive(alice, bob)\n')
    comp = Computation.from_textual(src)
    for fmt in sorted(ENC):
        enc, dec = ENC[fmt]
        back = dec(enc(comp))
        assert back.to_textual() == comp.to_textual(), fmt
        bits = back.operations[3].attrs["value"].value
        np.testing.assert_array_equal(bits, [[1, 0, 1], [1, 1, 0]])


def test_fused_operators_and_corrupt_input_are_rejected():
    comp = Computation.from_textual('x = Constant{value = Float64(1.0)}: () -> Float64 () @Host(a)\n')
    comp.operations[0].kind = "RingDotCross"
    with pytest.raises(RS.RustSerdeError):
        RS.to_rust_bincode(comp)
    good = Computation.from_textual('x = Constant{value = Float64(1.0)}: () -> Float64 () @Host(a)\n')
    for enc, dec in ENC.values():
        data = enc(good)
        with pytest.raises(RS.RustSerdeError):
            dec(data[:-3])
        with pytest.raises(RS.RustSerdeError):
            dec(data + b"\x00")
    bad = bytearray(RS.to_rust_bincode(good))
    bad[8 + 8 + 1] = 99  # operator variant index out of range
    with pytest.raises(RS.RustSerdeError):
        RS.from_rust_bincode(bytes(bad))


@pytest.mark.parametrize("fmt", ["bincode-rs", "msgpack-rs"])
def test_elk_compile_rust_layouts(tmp_path, fmt):
    src = os.path.join(REPO, "examples", "dot.moose")
    out = tmp_path / "dot.bin"
    assert elk.main(["compile", src, "-o", str(out), "-f", fmt, "-p", "typing"]) == 0
    back = tmp_path / "back.moose"
    assert elk.main(["compile", str(out), "-i", fmt, "-o", str(back), "-f", "textual",
                     "-p", "typing"]) == 0
    ref = Computation.from_textual(open(src).read())
    assert len(Computation.from_textual(back.read_text())) == len(ref)


def test_reference_fixed_constant_form(monkeypatch):
    """The reference prints a Fixed constant as Fixed(value, precision)
    (textual/parsing.rs:1556); both parsers read it (integral precision 0), and the Rust
    layout carries that one precision."""
    src = 'x = Constant{value = Fixed(1.5, 40)}: () -> Fixed () @Host(a)\n'
    for native in ("1", "0"):
        monkeypatch.setenv("MOOSEX_NATIVE_RUNTIME", native)
        c = Computation.from_textual(src)
        assert c.operations[0].attrs["value"].value == (1.5, 0, 40)
        data = RS.to_rust_bincode(c)
        assert data.endswith(struct.pack("<d", 1.5) + _u64(40) + _u64(0) + _u32(0) + _s("a"))
        assert RS.from_rust_bincode(data).to_textual() == c.to_textual()


@pytest.mark.parametrize("fmt", sorted(ENC))
def test_every_type_and_placement_round_trips(fmt):
    """All 66 Ty variants (with the TensorShape / TensorDType inners) in signatures, on all
    four placement kinds."""
    from moose_amd.ir.computation import Operation
    from moose_amd.ir.computation import Signature
    from moose_amd.ir.computation import placement_from
    from moose_amd.ir.types import SHAPE_KINDS
    from moose_amd.ir.types import TensorDType
    from moose_amd.ir.types import Ty

    tys = [Ty(n) for n in RS.TY_VARIANTS if n not in ("Shape", "Tensor")]
    tys += [Ty("Shape", k) for k in SHAPE_KINDS]
    tys += [Ty("Tensor", TensorDType(k, 3, 5) if k.startswith("Fixed") else TensorDType(k))
            for k in RS.DTYPE_VARIANTS]
    plcs = [placement_from("Host", ["a"]), placement_from("Replicated", ["a", "b", "c"]),
            placement_from("Additive", ["a", "b"]), placement_from("Mirrored3", ["a", "b", "c"])]
    ops = [Operation(f"op{i}", "Identity", [], plcs[i % 4], Signature((t,), t), {})
           for i, t in enumerate(tys)]
    comp = Computation(ops)
    enc, dec = ENC[fmt]
    back = dec(enc(comp))
    assert [(o.sig, o.placement) for o in back.operations] == [(o.sig, o.placement) for o in ops]
