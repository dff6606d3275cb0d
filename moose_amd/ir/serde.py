"""Binary serialisation of native-IR computations (msgpack).

Parity: reference ``Computation::{to,from}_msgpack`` / ``to_disk`` / ``from_disk``
(``moose/src/computation.rs:1815-1874``).  The encoding is our own compact msgpack
layout (operation tuples); numpy payloads travel as raw little-endian bytes.
"""
import msgpack
import numpy as np

from moose_amd.ir.computation import Computation
from moose_amd.ir.computation import Constant
from moose_amd.ir.computation import Operation
from moose_amd.ir.computation import Signature
from moose_amd.ir.computation import placement_from
from moose_amd.ir.types import Ty
from moose_amd.ir.types import TensorDType

_FORMAT = "moosex-ir-1"


def _enc_ty(t: Ty):
    if isinstance(t.inner, TensorDType):
        return [t.name, t.inner.kind, t.inner.integral_precision, t.inner.fractional_precision]
    return [t.name, t.inner]


def _dec_ty(x):
    if len(x) == 4:
        return Ty(x[0], TensorDType(x[1], x[2], x[3]))
    return Ty(x[0], x[1])


def _enc_attr(v):
    if isinstance(v, Constant):
        val = v.value
        if isinstance(val, np.ndarray):
            if val.dtype == object:
                payload = {"obj": [str(int(e)) for e in val.flatten()], "shape": list(val.shape)}
            else:
                payload = {"dt": val.dtype.str, "shape": list(val.shape), "b": val.tobytes()}
            return {"__c": v.kind, "nd": payload}
        if isinstance(val, tuple):
            val = list(val)
        return {"__c": v.kind, "v": _enc_attr(val)}
    if isinstance(v, tuple):
        return {"__t": [_enc_attr(x) for x in v]}
    if isinstance(v, list):
        return [_enc_attr(x) for x in v]
    if isinstance(v, int) and not isinstance(v, bool) and not -(1 << 63) <= v < (1 << 64):
        return {"__i": str(v)}  # ring constants / weights wider than msgpack ints
    return v


def _dec_attr(v):
    if isinstance(v, list):
        return [_dec_attr(x) for x in v]
    if isinstance(v, dict) and "__i" in v:
        return int(v["__i"])
    if isinstance(v, dict) and "__c" in v:
        if "nd" in v:
            p = v["nd"]
            if "obj" in p:
                arr = np.array([int(e) for e in p["obj"]], dtype=object).reshape(p["shape"])
            else:
                arr = np.frombuffer(p["b"], dtype=np.dtype(p["dt"])).reshape(p["shape"]).copy()
            return Constant(v["__c"], arr)
        val = _dec_attr(v["v"])
        if v["__c"] == "HostShape" or v["__c"] == "Fixed":
            val = tuple(val)
        return Constant(v["__c"], val)
    if isinstance(v, dict) and "__t" in v:
        return tuple(_dec_attr(x) for x in v["__t"])
    return v


def to_msgpack(comp: Computation) -> bytes:
    ops = []
    for op in comp.operations:
        plc = op.placement
        kind = type(plc).__name__.replace("Placement", "")
        ops.append(
            [
                op.name,
                op.kind,
                op.inputs,
                [kind, list(plc.owners)],
                [[_enc_ty(a) for a in op.sig.args], _enc_ty(op.sig.ret), op.sig.variadic],
                {k: _enc_attr(v) for k, v in op.attrs.items()},
            ]
        )
    return msgpack.packb({"format": _FORMAT, "ops": ops}, use_bin_type=True)


def from_msgpack(data: bytes) -> Computation:
    d = msgpack.unpackb(data, raw=False, strict_map_key=False)
    if d.get("format") != _FORMAT:
        raise ValueError("not a moosex IR msgpack payload")
    out = []
    for name, kind, inputs, (pk, owners), (args, ret, var), attrs in d["ops"]:
        out.append(
            Operation(
                name,
                kind,
                list(inputs),
                placement_from(pk, owners),
                Signature(tuple(_dec_ty(a) for a in args), _dec_ty(ret), bool(var)),
                {k: _dec_attr(v) for k, v in attrs.items()},
            )
        )
    return Computation(out)
