"""Shared helpers of the CLI tools: computation IO and argument-shape flags."""
from __future__ import annotations

from moose_amd.ir.computation import Computation

# msgpack / bincode: this framework's compact binary forms; msgpack-rs / bincode-rs: the
# reference's own NamedComputation bytes (moose_amd/ir/rust_serde.py)
FORMATS = ("textual", "msgpack", "bincode", "msgpack-rs", "bincode-rs")


def _rust(fmt):
    from moose_amd.ir import rust_serde

    if fmt == "msgpack-rs":
        return rust_serde.to_rust_msgpack, rust_serde.from_rust_msgpack
    return rust_serde.to_rust_bincode, rust_serde.from_rust_bincode


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
    if fmt in ("msgpack-rs", "bincode-rs"):
        with open(path, "rb") as f:
            return _rust(fmt)[1](f.read())
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
    if fmt in ("msgpack-rs", "bincode-rs"):
        if path is None:
            raise ValueError(f"{fmt} output needs --output")
        with open(path, "wb") as f:
            f.write(_rust(fmt)[0](comp))
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
