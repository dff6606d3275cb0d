"""Logical (placement-typed) values flowing through the interpreter.

Parity: the reference's ``AbstractTensor``/``FixedTensor``/``BoolTensor`` enums
(``moose/src/logical/mod.rs``, ``fixedpoint/mod.rs``, ``boolean/mod.rs``) -- a logical
tensor is Host-, Replicated- or Mirrored3-placed and carries its TensorDType.

Storage by dtype:

* host / mirrored: Float32/Float64 -> ``torch`` float tensor; Bool -> ``torch.bool``;
  Uint64 -> ``torch.int64`` (bit pattern); Fixed64/Fixed128 -> ring ``RT`` holding the
  encoded integers (scale 2^fractional_precision);
* replicated: Fixed -> arithmetic ``RepTensor`` over the dtype's ring; Bool -> boolean
  bit sharing; Uint64 -> arithmetic sharing over Z_2^64.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any
from typing import Optional

from moose_amd.ir.computation import HostPlacement
from moose_amd.ir.computation import Mirrored3Placement
from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ir.types import TensorDType


@dataclass
class LV:
    plc: Any  # HostPlacement | ReplicatedPlacement | Mirrored3Placement
    kind: str  # tensor | shape | string | unit | float | int | aeskey | aestensor | seed | key
    dtype: Optional[TensorDType]
    v: Any

    @property
    def is_host(self):
        return isinstance(self.plc, HostPlacement)

    @property
    def is_rep(self):
        return isinstance(self.plc, ReplicatedPlacement)

    @property
    def is_mir(self):
        return isinstance(self.plc, Mirrored3Placement)

    @property
    def host(self):
        return self.plc.owner


@dataclass
class MV:
    """Mirrored (public, replicated in the clear on 3 hosts) value.  ``v`` is the value
    (stacked session) or this party's copy (SPMD session, ``None`` off-placement)."""

    plc: Mirrored3Placement
    v: Any
