"""Minimal ONNX ``ModelProto`` reader (no ``onnx`` package needed).

Decodes the protobuf wire format directly for the subset of onnx.proto the predictors
use: ModelProto, GraphProto, NodeProto, AttributeProto, TensorProto, ValueInfoProto and
the tensor type/shape messages.  Decoded messages are plain objects whose attributes
follow the ONNX field names (``model.graph.node[i].op_type``, ``attr.floats``,
``tensor.raw_data`` ...), defaulting like protobuf (0 / "" / empty list).

Nothing in a model file is executed: bytes are only interpreted as numbers, strings and
nested messages.
"""
from __future__ import annotations

import struct
from typing import Dict
from typing import Tuple

import numpy as np

# field number -> (name, kind, repeated); kind: int | float | double | str | bytes | msg:<Name>
_SCHEMA: Dict[str, Dict[int, Tuple[str, str, bool]]] = {
    "ModelProto": {
        1: ("ir_version", "int", False), 2: ("producer_name", "str", False),
        3: ("producer_version", "str", False), 4: ("domain", "str", False),
        5: ("model_version", "int", False), 6: ("doc_string", "str", False),
        7: ("graph", "msg:GraphProto", False), 8: ("opset_import", "msg:OperatorSetIdProto", True),
    },
    "OperatorSetIdProto": {1: ("domain", "str", False), 2: ("version", "int", False)},
    "GraphProto": {
        1: ("node", "msg:NodeProto", True), 2: ("name", "str", False),
        5: ("initializer", "msg:TensorProto", True), 10: ("doc_string", "str", False),
        11: ("input", "msg:ValueInfoProto", True), 12: ("output", "msg:ValueInfoProto", True),
        13: ("value_info", "msg:ValueInfoProto", True),
    },
    "NodeProto": {
        1: ("input", "str", True), 2: ("output", "str", True), 3: ("name", "str", False),
        4: ("op_type", "str", False), 5: ("attribute", "msg:AttributeProto", True),
        6: ("doc_string", "str", False), 7: ("domain", "str", False),
    },
    "AttributeProto": {
        1: ("name", "str", False), 2: ("f", "float", False), 3: ("i", "int", False),
        4: ("s", "bytes", False), 5: ("t", "msg:TensorProto", False),
        6: ("g", "msg:GraphProto", False), 7: ("floats", "float", True),
        8: ("ints", "int", True), 9: ("strings", "bytes", True),
        10: ("tensors", "msg:TensorProto", True), 11: ("graphs", "msg:GraphProto", True),
        13: ("doc_string", "str", False), 20: ("type", "int", False),
        21: ("ref_attr_name", "str", False),
    },
    "TensorProto": {
        1: ("dims", "int", True), 2: ("data_type", "int", False), 4: ("float_data", "float", True),
        5: ("int32_data", "int", True), 6: ("string_data", "bytes", True),
        7: ("int64_data", "int", True), 8: ("name", "str", False), 9: ("raw_data", "bytes", False),
        10: ("double_data", "double", True), 11: ("uint64_data", "int", True),
        12: ("doc_string", "str", False),
    },
    "ValueInfoProto": {1: ("name", "str", False), 2: ("type", "msg:TypeProto", False),
                       3: ("doc_string", "str", False)},
    "TypeProto": {1: ("tensor_type", "msg:TypeProtoTensor", False)},
    "TypeProtoTensor": {1: ("elem_type", "int", False), 2: ("shape", "msg:TensorShapeProto", False)},
    "TensorShapeProto": {1: ("dim", "msg:Dimension", True)},
    "Dimension": {1: ("dim_value", "int", False), 2: ("dim_param", "str", False)},
}

# AttributeProto.type values
FLOAT, INT, STRING, TENSOR, GRAPH, FLOATS, INTS, STRINGS = 1, 2, 3, 4, 5, 6, 7, 8


class Message:
    def __init__(self, kind):
        self._kind = kind
        for _, (name, k, rep) in _SCHEMA[kind].items():
            if rep:
                setattr(self, name, [])
            elif k.startswith("msg:"):
                setattr(self, name, None)
            elif k in ("str",):
                setattr(self, name, "")
            elif k == "bytes":
                setattr(self, name, b"")
            elif k in ("float", "double"):
                setattr(self, name, 0.0)
            else:
                setattr(self, name, 0)

    def __repr__(self):
        n = getattr(self, "name", "")
        return f"<{self._kind} {n}>"


def _varint(buf, i):
    r = 0
    shift = 0
    while True:
        b = buf[i]
        i += 1
        r |= (b & 0x7F) << shift
        if not b & 0x80:
            return r, i
        shift += 7


def _signed64(v):
    return v - (1 << 64) if v >= (1 << 63) else v


def parse(kind: str, buf: bytes, start=0, end=None) -> Message:
    schema = _SCHEMA[kind]
    msg = Message(kind)
    i = start
    end = len(buf) if end is None else end
    while i < end:
        key, i = _varint(buf, i)
        field, wire = key >> 3, key & 7
        spec = schema.get(field)
        if wire == 0:
            v, i = _varint(buf, i)
            if spec:
                _set(msg, spec, _signed64(v))
        elif wire == 1:
            raw = buf[i:i + 8]
            i += 8
            if spec:
                _set(msg, spec, struct.unpack("<d", raw)[0] if spec[1] == "double"
                     else struct.unpack("<q", raw)[0])
        elif wire == 5:
            raw = buf[i:i + 4]
            i += 4
            if spec:
                _set(msg, spec, struct.unpack("<f", raw)[0] if spec[1] == "float"
                     else struct.unpack("<i", raw)[0])
        elif wire == 2:
            n, i = _varint(buf, i)
            chunk_end = i + n
            if spec:
                name, k, rep = spec
                if k.startswith("msg:"):
                    _set(msg, spec, parse(k[4:], buf, i, chunk_end))
                elif k == "str":
                    _set(msg, spec, bytes(buf[i:chunk_end]).decode("utf-8", errors="replace"))
                elif k == "bytes":
                    _set(msg, spec, bytes(buf[i:chunk_end]))
                elif rep:  # packed repeated scalars
                    data = bytes(buf[i:chunk_end])
                    if k == "float":
                        getattr(msg, name).extend(np.frombuffer(data, "<f4").tolist())
                    elif k == "double":
                        getattr(msg, name).extend(np.frombuffer(data, "<f8").tolist())
                    else:
                        j = 0
                        vals = getattr(msg, name)
                        while j < len(data):
                            v, j = _varint(data, j)
                            vals.append(_signed64(v))
            i = chunk_end
        else:
            raise ValueError(f"unsupported protobuf wire type {wire}")
    return msg


def _set(msg, spec, v):
    name, _, rep = spec
    if rep:
        getattr(msg, name).append(v)
    else:
        setattr(msg, name, v)


def load_model(f) -> Message:
    """``onnx.load_model`` equivalent for a path, file object or bytes."""
    if isinstance(f, (bytes, bytearray)):
        data = bytes(f)
    elif hasattr(f, "read"):
        data = f.read()
    else:
        with open(f, "rb") as fh:
            data = fh.read()
    return parse("ModelProto", data)


_NP = {1: np.float32, 2: np.uint8, 3: np.int8, 5: np.int16, 6: np.int32, 7: np.int64,
       9: np.bool_, 10: np.float16, 11: np.float64, 12: np.uint32, 13: np.uint64}


def to_array(t: Message) -> np.ndarray:
    """``onnx.numpy_helper.to_array`` equivalent."""
    dt = _NP.get(t.data_type)
    if dt is None:
        raise ValueError(f"unsupported tensor data type {t.data_type}")
    shape = tuple(t.dims)
    if t.raw_data:
        a = np.frombuffer(t.raw_data, dtype=np.dtype(dt).newbyteorder("<"))
    elif t.data_type == 1:
        a = np.asarray(t.float_data, dtype=np.float32)
    elif t.data_type == 11:
        a = np.asarray(t.double_data, dtype=np.float64)
    elif t.data_type in (6, 2, 3, 5, 9):
        a = np.asarray(t.int32_data, dtype=dt)
    elif t.data_type == 7:
        a = np.asarray(t.int64_data, dtype=np.int64)
    else:
        a = np.asarray(t.uint64_data, dtype=dt)
    return a.reshape(shape).astype(dt)


# ---------------------------------------------------------------------------
# encoding (the inverse of parse, for models built in Python -- e.g. the tutorial's
# sklearn logistic regression exported the way skl2onnx does, without skl2onnx)
# ---------------------------------------------------------------------------
def _enc_varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def serialize(msg: Message) -> bytes:
    out = bytearray()
    for field, (name, k, rep) in sorted(_SCHEMA[msg._kind].items()):
        val = getattr(msg, name)
        vals = val if rep else [val]
        if rep and not vals:
            continue
        if not rep and (val is None or val == "" or val == b"" or
                        (k in ("int", "float", "double") and val == 0)):
            continue
        if rep and k in ("int", "float", "double"):  # packed
            if k == "float":
                data = np.asarray(vals, dtype="<f4").tobytes()
            elif k == "double":
                data = np.asarray(vals, dtype="<f8").tobytes()
            else:
                data = b"".join(_enc_varint(int(v)) for v in vals)
            out += _enc_varint((field << 3) | 2) + _enc_varint(len(data)) + data
            continue
        for v in vals:
            if k.startswith("msg:"):
                data = serialize(v)
                out += _enc_varint((field << 3) | 2) + _enc_varint(len(data)) + data
            elif k in ("str", "bytes"):
                data = v.encode() if isinstance(v, str) else bytes(v)
                out += _enc_varint((field << 3) | 2) + _enc_varint(len(data)) + data
            elif k == "float":
                out += _enc_varint((field << 3) | 5) + struct.pack("<f", v)
            elif k == "double":
                out += _enc_varint((field << 3) | 1) + struct.pack("<d", v)
            else:
                out += _enc_varint(field << 3) + _enc_varint(int(v))
    return bytes(out)


def make(kind: str, **fields) -> Message:
    m = Message(kind)
    for k, v in fields.items():
        setattr(m, k, v)
    return m


def attr(name: str, value) -> Message:
    if isinstance(value, str):
        return make("AttributeProto", name=name, s=value.encode(), type=STRING)
    if isinstance(value, int):
        return make("AttributeProto", name=name, i=value, type=INT)
    if isinstance(value, float):
        return make("AttributeProto", name=name, f=value, type=FLOAT)
    value = list(value)
    if value and isinstance(value[0], str):
        return make("AttributeProto", name=name, strings=[v.encode() for v in value],
                    type=STRINGS)
    if value and isinstance(value[0], (int, np.integer)):
        return make("AttributeProto", name=name, ints=[int(v) for v in value], type=INTS)
    return make("AttributeProto", name=name, floats=[float(v) for v in value], type=FLOATS)


def sklearn_logistic_regression_model(coef, intercept, n_features: int) -> bytes:
    """The ONNX graph skl2onnx emits for a binary ``LogisticRegression``
    (ml-inference-with-onnx tutorial): a LinearClassifier (ai.onnx.ml) with both class
    rows ``[-w, w]``, ``post_transform = LOGISTIC``, then a Normalizer and a ZipMap."""
    w = np.asarray(coef, dtype=np.float64).reshape(-1)
    b = float(np.asarray(intercept).reshape(-1)[0])
    lc = make("NodeProto", input=["float_input"], output=["label", "probability_tensor"],
              name="LinearClassifier", op_type="LinearClassifier", domain="ai.onnx.ml",
              attribute=[attr("classlabels_ints", [0, 1]),
                         attr("coefficients", list(-w) + list(w)),
                         attr("intercepts", [-b, b]),
                         attr("multi_class", 0), attr("post_transform", "LOGISTIC")])
    norm = make("NodeProto", input=["probability_tensor"], output=["probabilities"],
                name="Normalizer", op_type="Normalizer", domain="ai.onnx.ml",
                attribute=[attr("norm", "L1")])
    zm = make("NodeProto", input=["probabilities"], output=["output_probability"],
              name="ZipMap", op_type="ZipMap", domain="ai.onnx.ml",
              attribute=[attr("classlabels_int64s", [0, 1])])
    shape = make("TensorShapeProto", dim=[make("Dimension", dim_param="N"),
                                          make("Dimension", dim_value=n_features)])
    inp = make("ValueInfoProto", name="float_input",
               type=make("TypeProto", tensor_type=make("TypeProtoTensor", elem_type=1,
                                                       shape=shape)))
    out = make("ValueInfoProto", name="label",
               type=make("TypeProto", tensor_type=make("TypeProtoTensor", elem_type=7)))
    graph = make("GraphProto", node=[lc, norm, zm], name="ONNX(LogisticRegression)",
                 input=[inp], output=[out])
    model = make("ModelProto", ir_version=8, producer_name="skl2onnx",
                 producer_version="1.13", domain="ai.onnx", graph=graph,
                 opset_import=[make("OperatorSetIdProto", domain="", version=15),
                               make("OperatorSetIdProto", domain="ai.onnx.ml", version=1)])
    return serialize(model)
