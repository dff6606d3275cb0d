"""Operations of the eDSL IR (``pymoose.computation.operations``).

The reference spells out 46 dataclasses by hand
(``pymoose/pymoose/computation/operations.py``); here they are generated from a
single table of ``(class name, extra attribute fields)`` so that the tracer, the
msgpack codec and the converter to the native IR all read the same table.
"""
from dataclasses import dataclass
from dataclasses import field
from dataclasses import make_dataclass
from typing import Any
from typing import Dict

from moose_amd.computation import types as ty


@dataclass
class OpSignature:
    input_types: Dict[str, ty.ValueType]
    return_type: ty.ValueType


@dataclass(init=False)
class Operation:
    name: str
    inputs: Dict[str, str]
    placement_name: str
    signature: OpSignature

    @classmethod
    def identifier(cls):
        return cls.__name__

    @property
    def return_type(self):
        return self.signature.return_type


# (class name, [extra attribute names]) -- order matters for positional construction
OPERATION_TABLE = [
    ("AbsOperation", []),
    ("AddNOperation", []),
    ("AddOperation", []),
    ("ArgmaxOperation", ["axis", "upmost_index"]),
    ("AtLeast2DOperation", ["to_column_vector"]),
    ("BitwiseAndOperation", []),
    ("BitwiseOrOperation", []),
    ("CastOperation", []),
    ("ConcatenateOperation", ["axis"]),
    ("ConstantOperation", ["value"]),
    ("DecryptOperation", []),
    ("DivOperation", []),
    ("DotOperation", []),
    ("ExpandDimsOperation", ["axis"]),
    ("ExpOperation", []),
    ("GreaterOperation", []),
    ("IdentityOperation", []),
    ("IndexAxisOperation", ["axis", "index"]),
    ("InputOperation", []),
    ("InverseOperation", []),
    ("LessOperation", []),
    ("LoadOperation", []),
    ("LogOperation", []),
    ("Log2Operation", []),
    ("MaximumOperation", []),
    ("MeanOperation", ["axis"]),
    ("MulOperation", []),
    ("MuxOperation", []),
    ("OnesOperation", []),
    ("ZerosOperation", []),
    ("OutputOperation", ["tag"]),
    ("SigmoidOperation", []),
    ("ReluOperation", []),
    ("SelectOperation", ["axis"]),
    ("SoftmaxOperation", ["axis", "upmost_index"]),
    ("ReshapeOperation", []),
    ("SaveOperation", []),
    ("ShapeOperation", []),
    ("SliceOperation", ["begin", "end"]),
    ("StridedSliceOperation", ["slices"]),
    ("SqueezeOperation", ["axis"]),
    ("SqrtOperation", []),
    ("SubOperation", []),
    ("SumOperation", ["axis"]),
    ("TransposeOperation", []),
]

OPERATION_CLASSES = {}
for _cls_name, _extras in OPERATION_TABLE:
    _fields = [
        ("name", str),
        ("inputs", Dict[str, str]),
        ("placement_name", str),
        ("signature", OpSignature),
    ] + [(e, Any, field(default=None)) for e in _extras]
    _cls = make_dataclass(_cls_name, _fields, bases=(Operation,))
    _cls.__module__ = __name__
    OPERATION_CLASSES[_cls_name] = _cls
    globals()[_cls_name] = _cls

del _cls_name, _extras, _fields, _cls
