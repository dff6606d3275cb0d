"""``MooseComputation``: a compiled (native-IR) computation handle.

Parity: reference ``pymoose/src/bindings.rs:332-401`` (``from_bytes`` / ``to_bytes`` /
``from_disk`` / ``to_disk`` / ``from_textual`` / ``to_textual``).  The byte format is
this framework's IR msgpack (``moose_amd.ir.serde``); ``from_bytes`` also accepts the
pymoose eDSL msgpack produced by ``moose_amd.computation.utils.serialize_computation``.
"""
from __future__ import annotations

from moose_amd.ir.computation import Computation


class MooseComputation:
    def __init__(self, native: Computation):
        self.native = native

    @classmethod
    def from_py(cls, computation, fixedpoint_ring: int = 128):
        from moose_amd.runtime.local import to_native

        return cls(to_native(computation, fixedpoint_ring))

    @classmethod
    def from_bytes(cls, data: bytes):
        from moose_amd.runtime.local import to_native

        return cls(to_native(bytes(data)))

    def to_bytes(self) -> bytes:
        return self.native.to_msgpack()

    @classmethod
    def from_disk(cls, path):
        return cls(Computation.from_disk(path))

    def to_disk(self, path):
        self.native.to_disk(path)

    @classmethod
    def from_textual(cls, text: str):
        return cls(Computation.from_textual(text))

    def to_textual(self) -> str:
        return self.native.to_textual()

    def __len__(self):
        return len(self.native.operations)

    def __repr__(self):
        return f"MooseComputation({len(self)} operations)"
