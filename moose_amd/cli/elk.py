"""``elk``: compile computations and print graph statistics.

Parity: reference ``moose/src/bin/elk/main.rs:11-276``::

    elk compile INPUT [-o OUT] [-i FORMAT] [-f FORMAT] [-p pass,pass]
        (FORMAT: textual, msgpack, bincode, or the reference's own msgpack-rs / bincode-rs)
                      [--arg-shape name=3,4 ...]
    elk stats op-hist  INPUT [--by-placement]
    elk stats op-count INPUT [--by-placement]
    elk stats out-degree INPUT [--by-operator]

Without ``--arg-shape`` lowering is shape-polymorphic, as in the reference (input shapes
are read at run time through ``Shape`` operations; one plan serves every input size).
``--arg-shape`` specialises the plan to fixed input shapes: static shapes throughout, the
form a hipGraph capture replays, and the only form for protocols whose structure depends
on a size (argmax / softmax over a dynamic axis).
"""
from __future__ import annotations

import argparse
import sys
from collections import Counter

from moose_amd.cli.common import FORMATS
from moose_amd.cli.common import parse_arg_shapes
from moose_amd.cli.common import read_computation
from moose_amd.cli.common import write_computation


def _placement_key(op):
    return op.placement.to_textual()


def op_hist(comp, by_placement=False):
    c = Counter((op.kind, _placement_key(op)) if by_placement else op.kind
                for op in comp.operations)
    lines = []
    for k, n in sorted(c.items(), key=lambda kv: (-kv[1], str(kv[0]))):
        lines.append(f"{n} {k[0]} {k[1]}" if by_placement else f"{n} {k}")
    return lines


def op_count(comp, by_placement=False):
    if not by_placement:
        return [str(len(comp.operations))]
    c = Counter(_placement_key(op) for op in comp.operations)
    return [f"{n} {k}" for k, n in sorted(c.items(), key=lambda kv: (-kv[1], kv[0]))]


def out_degree(comp, by_operator=False):
    deg = Counter()
    for op in comp.operations:
        for i in op.inputs:
            deg[i] += 1
    kinds = {op.name: op.kind for op in comp.operations}
    if by_operator:
        hist = Counter((kinds[n], deg.get(n, 0)) for n in kinds)
        return [f"{n} {k} {d}" for (k, d), n in sorted(hist.items(), key=lambda kv: (kv[0][0], kv[0][1]))]
    hist = Counter(deg.get(n, 0) for n in kinds)
    return [f"{d} {n}" for d, n in sorted(hist.items())]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="elk", description="Moose (MI355X) compiler CLI")
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("compile")
    c.add_argument("input")
    c.add_argument("-o", "--output")
    c.add_argument("-i", "--input-format", default="textual", choices=FORMATS)
    c.add_argument("-f", "--output-format", default="textual", choices=FORMATS)
    c.add_argument("-p", "--passes")
    c.add_argument("--arg-shape", action="append", default=[])
    c.add_argument("--fixedpoint-ring", type=int, default=128, choices=(64, 128))
    s = sub.add_parser("stats")
    ss = s.add_subparsers(dest="stat", required=True)
    for name, flag in (("op-hist", "--by-placement"), ("op-count", "--by-placement"),
                       ("out-degree", "--by-operator")):
        p = ss.add_parser(name)
        p.add_argument("input")
        p.add_argument("-i", "--input-format", default="textual", choices=FORMATS)
        p.add_argument(flag, action="store_true")
    a = ap.parse_args(argv)
    if a.cmd == "compile":
        from moose_amd.compiler import passes as P

        comp = read_computation(a.input, a.input_format)
        names = [p for p in a.passes.split(",") if p] if a.passes is not None else None
        comp = P.compile(comp, names, arg_specs=parse_arg_shapes(a.arg_shape),
                         fixedpoint_ring=a.fixedpoint_ring)
        write_computation(comp, a.output, a.output_format)
        return 0
    comp = read_computation(a.input, a.input_format)
    if a.stat == "op-hist":
        lines = op_hist(comp, a.by_placement)
    elif a.stat == "op-count":
        lines = op_count(comp, a.by_placement)
    else:
        lines = out_degree(comp, a.by_operator)
    sys.stdout.write("\n".join(lines) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
