"""``elk_compiler.compile_computation`` (reference ``pymoose/src/bindings.rs:403-419``):
compile a serialized computation with the named passes (default pipeline when
``passes`` is None; ``[]`` only converts to the native IR)."""
from __future__ import annotations

from moose_amd.compiler import passes as _passes
from moose_amd.compiler.api import MooseComputation


def compile_computation(computation, passes=None, arg_specs=None, fixedpoint_ring: int = 128):
    mc = (computation if isinstance(computation, MooseComputation)
          else MooseComputation.from_py(computation, fixedpoint_ring)
          if not isinstance(computation, (bytes, bytearray))
          else MooseComputation.from_bytes(computation))
    comp = _passes.compile(mc.native, passes, arg_specs=arg_specs, fixedpoint_ring=fixedpoint_ring)
    return MooseComputation(comp)
