"""Shared helpers of the CLI tools: computation IO and argument-shape flags."""
from __future__ import annotations

from moose_amd.ir.computation import Computation

FORMATS = ("textual", "msgpack", "bincode")


def read_computation(path, fmt="textual") -> Computation:
    if fmt == "textual":
        with open(path) as f:
            return Computation.from_textual(f.read())
    if fmt == "msgpack":
        with open(path, "rb") as f:
            return Computation.from_msgpack(f.read())
    if fmt == "bincode":
        with open(path, "rb") as f:
            return Computation.from_bincode(f.read())
    raise ValueError(f"unsupported computation format {fmt!r}")


def write_computation(comp: Computation, path, fmt="textual"):
    if fmt == "textual":
        data = comp.to_textual() + "\n"
        if path is None:
            print(data, end="")
        else:
            with open(path, "w") as f:
                f.write(data)
        return
    if fmt == "msgpack":
        if path is None:
            raise ValueError("msgpack output needs --output")
        with open(path, "wb") as f:
            f.write(comp.to_msgpack())
        return
    if fmt == "bincode":
        if path is None:
            raise ValueError("bincode output needs --output")
        with open(path, "wb") as f:
            f.write(comp.to_bincode())
        return
    raise ValueError(f"unsupported computation format {fmt!r}")


def parse_arg_shapes(items):
    """``["x=3,4", "y=4x2"]`` -> ``{"x": (3, 4), "y": (4, 2)}``."""
    specs = {}
    for it in items or []:
        name, _, dims = it.partition("=")
        dims = dims.replace("x", ",")
        specs[name] = tuple(int(d) for d in dims.split(",") if d.strip())
    return specs
