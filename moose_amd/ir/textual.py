"""Textual ``.moose`` format: parser and printer.

Parity: reference ``moose/src/textual/parsing.rs`` (verbose parser :61, parallel
parser :83-117, placement :190, constant literals :608, printers :1135+).  One op per
assignment::

    name = Kind{attr = value, ...}: (T1, T2) -> T (in1, in2) @Host(alice)

The parser is a regex-driven cursor parser; ``parse_computation(parallel=True)``
splits large sources at line breaks and parses the chunks in a process pool (the
analogue of the reference's rayon ``parallel_parse_computation``).  The native C++
parser (``csrc/runtime/textual.cpp``, chunks on native threads) is used when the
runtime extension is available; this Python one is its oracle.
"""
from __future__ import annotations

import os
import re
from concurrent.futures import ProcessPoolExecutor
from typing import List

import numpy as np

from moose_amd import errors
from moose_amd.ir.computation import Computation
from moose_amd.ir.computation import Constant
from moose_amd.ir.computation import Operation
from moose_amd.ir.computation import Signature
from moose_amd.ir.computation import TENSOR_CONSTANT_NP
from moose_amd.ir.computation import _float_literal
from moose_amd.ir.computation import _quote
from moose_amd.ir.computation import placement_from
from moose_amd.ir.operators import ALL_OPERATORS
from moose_amd.ir.operators import DEFAULT_RETURN
from moose_amd.ir.operators import OPERATOR_ALIASES
from moose_amd.ir.types import Ty

_WS = re.compile(r"(?:\s+|//[^\n\r]*)*")
_IDENT = re.compile(r"[A-Za-z0-9_]+")
_NUMBER = re.compile(r"[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?|[-+]?inf|NaN")
_INT = re.compile(r"[-+]?\d+")
_HEX = re.compile(r"[0-9a-fA-F]+")
_STRING = re.compile(r'"((?:[^"\\]|\\.)*)"')
_TYPE = re.compile(r"[A-Za-z0-9]+(?:<[^>]*>)?")


class ParseError(errors.MalformedComputation, ValueError):
    pass


class _Cursor:
    __slots__ = ("s", "i")

    def __init__(self, s, i=0):
        self.s = s
        self.i = i

    def ws(self):
        self.i = _WS.match(self.s, self.i).end()

    def peek(self, lit):
        self.ws()
        return self.s.startswith(lit, self.i)

    def eat(self, lit):
        if self.peek(lit):
            self.i += len(lit)
            return True
        return False

    def expect(self, lit):
        if not self.eat(lit):
            self.fail(f"expected {lit!r}")

    def match(self, rx, what):
        self.ws()
        m = rx.match(self.s, self.i)
        if not m:
            self.fail(f"expected {what}")
        self.i = m.end()
        return m

    def fail(self, msg):
        line = self.s.count("\n", 0, self.i) + 1
        snippet = self.s[self.i : self.i + 60].split("\n")[0]
        raise ParseError(f"line {line}: {msg} at {snippet!r}")

    def at_end(self):
        self.ws()
        return self.i >= len(self.s)


# ---------------------------------------------------------------------------
# values
# ---------------------------------------------------------------------------
def _parse_nested(c: _Cursor, scalar):
    if c.eat("["):
        items = []
        if not c.eat("]"):
            while True:
                items.append(_parse_nested(c, scalar))
                if c.eat("]"):
                    break
                c.expect(",")
        return items
    return scalar(c)


def _num(c):
    m = c.match(_NUMBER, "number").group(0)
    if m in ("inf", "+inf"):
        return float("inf")
    if m == "-inf":
        return float("-inf")
    if m == "NaN":
        return float("nan")
    if re.fullmatch(r"[-+]?\d+", m):
        return int(m)
    return float(m)


def _parse_constant_literal(c: _Cursor, kind: str) -> Constant:
    c.expect("(")
    if kind in TENSOR_CONSTANT_NP:
        nested = _parse_nested(c, _num)
        npd = TENSOR_CONSTANT_NP[kind]
        if npd is object:
            arr = np.array(nested, dtype=object)
        else:
            arr = np.array(nested, dtype=npd)
        val = Constant(kind, arr)
    elif kind == "HostShape":
        val = Constant(kind, tuple(int(x) for x in _parse_nested(c, _num)))
    elif kind in ("HostString", "String"):
        m = c.match(_STRING, "string")
        val = Constant("HostString", _unquote(m.group(1)))
    elif kind in ("HostSeed", "HostPrfKey", "Seed", "PrfKey"):
        if c.peek("["):
            raw = bytes(int(x) for x in _parse_nested(c, _num))
        else:
            raw = bytes.fromhex(c.match(_HEX, "hex").group(0))
        val = Constant({"Seed": "HostSeed", "PrfKey": "HostPrfKey"}.get(kind, kind), raw)
    elif kind in ("Ring64", "Ring128", "Bit"):
        val = Constant(kind, int(c.match(_INT, "integer").group(0)))
    elif kind in ("Float32", "Float64"):
        val = Constant(kind, float(_num(c)))
    elif kind == "Fixed":
        v = float(_num(c))
        c.expect(",")
        i = int(_num(c))
        if c.eat(","):
            f = int(_num(c))
        else:  # the reference's Fixed(value, precision) (textual/parsing.rs:1556)
            i, f = 0, i
        val = Constant("Fixed", (v, i, f))
    else:
        c.fail(f"unknown constant kind {kind}")
    c.expect(")")
    return val


def _unquote(s):
    return s.replace('\\"', '"').replace("\\\\", "\\")


def _parse_value(c: _Cursor, kind: str):
    if kind == "key":
        if c.peek("["):
            return bytes(int(x) for x in _parse_nested(c, _num))
        h = c.match(_HEX, "hex key").group(0)
        return bytes.fromhex(h.rjust(32, "0"))
    if kind == "str":
        return _unquote(c.match(_STRING, "string").group(1))
    if kind == "bool":
        w = c.match(_IDENT, "bool").group(0)
        return w == "true"
    if kind in ("int", "opt_int"):
        if c.peek("None"):
            c.eat("None")
            return None
        return int(c.match(_INT, "integer").group(0))
    if kind in ("ints", "opt_ints"):
        if kind == "opt_ints" and c.eat("None"):
            return None
        return [int(x) for x in _parse_nested(c, _num)]
    if kind == "const":
        if c.peek('"'):
            return Constant("HostString", _unquote(c.match(_STRING, "string").group(1)))
        name = c.match(_IDENT, "constant kind").group(0)
        return _parse_constant_literal(c, name)
    if kind == "slice":
        if c.eat("["):  # multi-axis slice: [{start = ..}, {..}] (one element per axis)
            out = []
            while not c.eat("]"):
                out.append(_parse_value(c, "slice"))
                c.eat(",")
            return out
        c.expect("{")
        d = {"start": 0, "end": None, "step": None}
        while not c.eat("}"):
            k = c.match(_IDENT, "slice field").group(0)
            c.expect("=")
            d[k] = None if c.eat("None") else int(c.match(_INT, "integer").group(0))
            c.eat(",")
        return (d["start"], d["end"], d["step"])
    raise AssertionError(kind)


def _parse_type(c: _Cursor) -> Ty:
    c.ws()
    m = _TYPE.match(c.s, c.i)
    if not m:
        c.fail("expected a type")
    txt = m.group(0)
    # Tensor<Fixed128(24, 40)> contains no '>' before the end, so the regex suffices
    c.i = m.end()
    try:
        return Ty.from_textual(txt)
    except ValueError as e:
        c.fail(str(e))


def _parse_signature(c: _Cursor):
    if c.eat("["):
        t = _parse_type(c)
        c.expect("]")
        c.expect("->")
        return Signature((t,), _parse_type(c), True)
    c.expect("(")
    args = []
    if not c.eat(")"):
        while True:
            args.append(_parse_type(c))
            if c.eat(")"):
                break
            c.expect(",")
    c.expect("->")
    return Signature(tuple(args), _parse_type(c))


def _parse_operation(c: _Cursor) -> Operation:
    name = c.match(_IDENT, "identifier").group(0)
    c.expect("=")
    kind = c.match(_IDENT, "operator name").group(0)
    kind = OPERATOR_ALIASES.get(kind, kind)
    schema = ALL_OPERATORS.get(kind)
    if schema is None:
        c.fail(f"unknown operator {kind}")
    kinds = dict(schema)
    attrs = {}
    if c.eat("{"):
        while not c.eat("}"):
            an = c.match(_IDENT, "attribute name").group(0)
            c.expect("=")
            if an not in kinds:
                c.fail(f"unknown attribute {an} for {kind}")
            attrs[an] = _parse_value(c, kinds[an])
            c.eat(",")
    for an, ak in schema:
        if an not in attrs:
            if ak in ("opt_int", "opt_ints"):
                attrs[an] = None
            elif kind == "Output" and an == "tag":
                attrs[an] = name  # older files omit the tag (examples/test.moose)
            elif kind == "Input" and an == "arg_name":
                attrs[an] = name
            else:
                c.fail(f"missing attribute {an} for {kind}")
    if c.eat(":"):
        sig = _parse_signature(c)
    elif kind in DEFAULT_RETURN:
        sig = Signature((), Ty(DEFAULT_RETURN[kind]))
    else:
        c.fail("expected a type signature")
    inputs: List[str] = []
    if c.eat("("):
        if not c.eat(")"):
            while True:
                inputs.append(c.match(_IDENT, "input name").group(0))
                if c.eat(")"):
                    break
                c.expect(",")
    c.expect("@")
    pk = c.match(_IDENT, "placement kind").group(0)
    c.expect("(")
    owners = []
    while True:
        owners.append(c.match(_IDENT, "role").group(0))
        if c.eat(")"):
            break
        c.expect(",")
    try:
        plc = placement_from(pk, owners)
    except (KeyError, ValueError) as e:
        c.fail(str(e))
    return Operation(name, kind, inputs, plc, sig, attrs)


def _parse_chunk(source: str) -> List[Operation]:
    c = _Cursor(source)
    ops = []
    while not c.at_end():
        ops.append(_parse_operation(c))
    return ops


def parse_computation(source: str, parallel: bool = True, chunks: int = 8) -> Computation:
    from moose_amd.runtime import native_rt

    if native_rt.enabled():
        try:
            return native_rt.parse(source, threads=chunks if parallel else 1)
        except native_rt.mod().NativeParseError as e:
            raise ParseError(str(e)) from None
        except ValueError as e:  # bad type / placement text
            raise ParseError(str(e)) from None
    return parse_computation_py(source, parallel, chunks)


def parse_computation_py(source: str, parallel: bool = True, chunks: int = 8) -> Computation:
    """Pure-Python parser (oracle for the native one; ``MOOSEX_NATIVE_RUNTIME=0``)."""
    if not parallel or len(source) < 2_000_000:
        return Computation(_parse_chunk(source))
    # split at line breaks into `chunks` parts (reference parsing.rs:83-117)
    parts, left, step = [], 0, len(source) // chunks
    for _ in range(chunks):
        right = min(len(source), left + step)
        nl = source.find("\n", right)
        right = len(source) if nl < 0 else nl + 1
        if right > left:
            parts.append(source[left:right])
        left = right
    if left < len(source):
        parts.append(source[left:])
    workers = min(len(parts), os.cpu_count() or 1)
    with ProcessPoolExecutor(max_workers=workers) as ex:
        results = list(ex.map(_parse_chunk, parts))
    return Computation([op for r in results for op in r])


# ---------------------------------------------------------------------------
# printer
# ---------------------------------------------------------------------------
def _print_value(v, kind):
    if kind == "key":
        return bytes(v).hex()
    if kind == "str":
        return _quote(v)
    if kind == "bool":
        return "true" if v else "false"
    if kind in ("int", "opt_int"):
        return str(int(v))
    if kind in ("ints", "opt_ints"):
        return "[" + ", ".join(str(int(x)) for x in v) + "]"
    if kind == "const":
        return v.to_textual()
    if kind == "slice":
        if isinstance(v, list):
            if len(v) == 1:
                v = v[0]
            else:
                return "[" + ", ".join(_print_value(e, "slice") for e in v) + "]"
        start, end, step = v
        s = f"{{start = {start}"
        if end is not None:
            s += f", end = {end}"
        if step is not None:
            s += f", step = {step}"
        return s + "}"
    raise AssertionError(kind)


def print_operation(op: Operation) -> str:
    schema = ALL_OPERATORS[op.kind]
    head = f"{op.name} = {op.kind}"
    if schema:
        parts = [
            f"{an} = {_print_value(op.attrs[an], ak)}"
            for an, ak in schema
            if op.attrs.get(an) is not None
        ]
        head += "{" + ", ".join(parts) + "}"
    return (
        f"{head}: {op.sig.to_textual()} ({', '.join(op.inputs)}) "
        f"{op.placement.to_textual()}"
    )


def print_computation(comp: Computation) -> str:
    return "\n".join(print_operation(op) for op in comp.operations)


__all__ = ["parse_computation", "print_computation", "print_operation", "ParseError",
           "_float_literal"]
