"""Executor for lowered (host-only) computations.

Parity: the reference runs compiled graphs with ``AsyncExecutor`` / ``TestSyncExecutor``
(``execution/asynchronous.rs:557-632``, ``execution/synchronous.rs:326-369``) and
``dasher`` (``bin/dasher/main.rs``) simulates all roles of a compiled computation in one
process.  Here every host operation is one primitive from
:mod:`moose_amd.runtime.prims` (ring kernels are the gfx950 HIP kernels), executed in
topological order.

* single process (``GraphExecutor.run``): all identities on one device; ``Send`` parks
  the value under its rendezvous key, the matching ``Receive`` picks it up;
* one process per identity (``identity=``/``transport=``): the process runs only its
  own operations.  Every process walks the same topological order and performs each
  Send/Receive pair at the position of the ``Send``, so the point-to-point messages of
  any two processes are matched by order (RCCL has no tags) -- the receiver parks the
  value until its ``Receive`` runs.
"""
from __future__ import annotations

import os
from typing import Dict
from typing import Optional

import numpy as np
import torch

from moose_amd import errors
from moose_amd.compiler.symbolic import bits_of_ty
from moose_amd.ir.computation import Computation
from moose_amd.ir.computation import Constant
from moose_amd.ops import ring as R
from moose_amd.runtime.prims import PRIMS

_NEEDS_BITS = {"Fill", "AddConst", "SampleSeeded", "Sample", "RingFixedpointEncode",
               "RingInject", "RingCast"}
_NEEDS_DEVICE = {"Fill", "SampleSeeded", "Sample", "Zeros", "Ones"}
# torch dtype of each plaintext host tensor type: unsigned types wider than 8 bits travel in
# a signed dtype (u16 -> i32 and u32 -> i64 widened, exact; u64 as its 64-bit pattern)
_TY_DTYPE = {"HostFloat64Tensor": torch.float64, "HostFloat32Tensor": torch.float32,
             "HostUint64Tensor": torch.int64, "HostInt64Tensor": torch.int64,
             "HostInt32Tensor": torch.int32, "HostInt16Tensor": torch.int16,
             "HostInt8Tensor": torch.int8, "HostUint8Tensor": torch.uint8,
             "HostUint16Tensor": torch.int32, "HostUint32Tensor": torch.int64,
             "HostBitTensor": torch.bool, "HostBoolTensor": torch.bool}


class GraphExecutionError(errors.KernelError):
    pass


def constant_value(c: Constant, device):
    k, v = c.kind, c.value
    if k == "HostRing64Tensor":
        return R.from_ints(np.asarray(v, dtype=object), 64, device)
    if k == "HostRing128Tensor":
        return R.from_ints(np.asarray(v, dtype=object), 128, device)
    if k == "HostBitTensor":
        return R.RT(torch.as_tensor(np.asarray(v, dtype=np.uint8), device=device), 1)
    if k in _TY_DTYPE and k not in ("HostBitTensor", "HostBoolTensor"):
        from moose_amd.runtime.interpreter import numpy_to_torch

        return numpy_to_torch(np.asarray(v), device).to(_TY_DTYPE[k])
    if k == "HostShape":
        return tuple(int(d) for d in v)
    if k in ("HostString", "HostSeed", "HostPrfKey"):
        return v
    if k in ("Ring64", "Ring128", "Bit"):
        return int(v)
    if k in ("Float32", "Float64"):
        return torch.tensor(float(v), dtype=torch.float64, device=device)
    raise GraphExecutionError(f"unsupported constant kind {k}")


def _attr_value(v):
    if isinstance(v, Constant):
        return int(v.value) if v.kind in ("Ring64", "Ring128", "Bit") else v.value
    return v


class GraphExecutor:
    def __init__(self, device="cpu", storage: Optional[Dict[str, dict]] = None,
                 identity: Optional[str] = None, transport=None, role_ranks=None,
                 workers: Optional[int] = None, timeout_s: Optional[float] = None):
        self.device = torch.device(device)
        self.storage = storage if storage is not None else {}
        self.identity = identity
        self.tr = transport
        self.role_ranks = role_ranks or {}
        self.workers = workers
        self.timeout_s = -1.0 if timeout_s is None else float(timeout_s)
        self.last_run_stats = None

    def _native_dataflow(self) -> bool:
        """Native scheduler for in-process runs and TCP-networked identities; RCCL runs
        keep the ordered walk (RCCL matches messages by order, not by key)."""
        from moose_amd.runtime import native_rt

        if os.environ.get("MOOSEX_DATAFLOW", "1") == "0" or not native_rt.enabled():
            return False
        if self.identity is None:
            return True
        from moose_amd.runtime.dataflow import TcpTransport

        return isinstance(self.tr, TcpTransport)

    def run(self, comp: Computation, arguments: Optional[dict] = None) -> dict:
        from moose_amd.runtime.interpreter import numpy_to_torch

        arguments = arguments or {}
        if self._native_dataflow():
            from moose_amd.runtime.dataflow import run_dataflow

            return run_dataflow(self, comp, arguments, self.workers, self.timeout_s)
        comp = comp.toposorted()
        self._used = set()
        env: Dict[str, object] = {}
        parked: Dict[bytes, object] = {}
        outputs = {}
        receivers = {bytes(op.attrs["rendezvous_key"]): op for op in comp.operations
                     if op.kind == "Receive"}
        me = self.identity
        for op in comp.operations:
            host = op.placement.owner
            if op.kind == "Send":
                key = bytes(op.attrs["rendezvous_key"])
                dst = op.attrs["receiver"]
                if key in parked or key in self._used:
                    # each (session, rendezvous key) is sent and received exactly once
                    raise GraphExecutionError(f"{op.name}: duplicate send for rendezvous key "
                                              f"{key.hex()}")
                if me is None:
                    parked[key] = env[op.inputs[0]]
                elif me == host:
                    self.tr.send(env[op.inputs[0]], self.role_ranks[dst])
                elif me == dst:
                    parked[key] = self.tr.recv(self.role_ranks[host], device=self.device)
                continue
            if me is not None and host != me:
                continue
            try:
                env[op.name] = self._exec(op, env, parked, arguments, outputs, receivers,
                                          numpy_to_torch)
            except GraphExecutionError:
                raise
            except Exception as e:
                raise GraphExecutionError(f"{op.name} = {op.kind} @ {host} failed: {e}") from e
        return outputs

    def _exec(self, op, env, parked, arguments, outputs, receivers, numpy_to_torch):
        kind = op.kind
        host = op.placement.owner
        vals = [env[i] for i in op.inputs]
        attrs = {k: _attr_value(v) for k, v in op.attrs.items()}
        if kind == "Constant":
            return constant_value(op.attrs["value"], self.device)
        if kind == "Input":
            name = attrs["arg_name"]
            if op.sig.ret.name == "HostUnit":
                return None
            if name not in arguments:
                raise GraphExecutionError(f"missing argument {name}")
            a = arguments[name]
            if isinstance(a, (str, bytes)) or op.sig.ret.name in ("HostString", "HostShape"):
                return a if not isinstance(a, list) else tuple(a)  # non-tensor arguments
            t = a.to(self.device) if isinstance(a, torch.Tensor) else numpy_to_torch(np.asarray(a), self.device)
            bits = bits_of_ty(op.sig.ret)
            if bits is not None and not isinstance(a, R.RT):
                return R.RT(t, bits)
            return t
        if kind == "Output":
            outputs[attrs.get("tag") or op.name] = vals[0]
            return vals[0]
        if kind == "Receive":
            key = bytes(attrs["rendezvous_key"])
            if key not in parked:
                raise GraphExecutionError(f"receive {op.name}: no value for its rendezvous key"
                                          + (" (already received)" if key in self._used else ""))
            self._used.add(key)
            return parked.pop(key)
        if kind == "PrfKeyGen":
            return os.urandom(16)
        if kind == "Save":
            key, val = vals
            self.storage.setdefault(host, {})[key] = val
            return None
        if kind == "Load":
            key = vals[0]
            return self.storage[host][key]
        if kind in ("RingMulCross", "BitAndCross", "RingDotCross"):
            return _cross(kind, *vals)
        return run_host_prim(op, vals, attrs, self.device)


def run_host_prim(op, vals, attrs, device):
    """One host-level operation as its primitive (shared with the interpreter's
    dialect-level fallback)."""
    kind = op.kind
    if kind in ("RingMulCross", "BitAndCross", "RingDotCross"):
        return _cross(kind, *vals)
    prim = PRIMS.get(kind)
    if prim is None:
        raise GraphExecutionError(f"no host kernel for {kind}")
    if kind == "Select":  # IR operands (index, x); the primitive takes (x, index)
        vals = [vals[1], vals[0]]
    elif kind == "Broadcast" and len(vals) == 2 and isinstance(vals[0], tuple):
        vals = [vals[1], vals[0]]  # IR (shape, x) as the reference's (kernels/mod.rs:230)
    return prim.impl(0, *vals, **prim_attrs(op, attrs, device))


def prim_attrs(op, attrs, device):
    """Keyword arguments of ``op``'s primitive: IR attributes plus the ring width /
    device / dtype its signature implies, minus IR-only attributes."""
    kind = op.kind
    prim = PRIMS[kind]
    attrs = dict(attrs)
    bits = bits_of_ty(op.sig.ret)
    if kind in _NEEDS_BITS:
        attrs["bits"] = bits
    if kind in _NEEDS_DEVICE:
        attrs["device"] = device
    if kind in ("Cast", "Zeros", "Ones", "RingFixedpointDecode"):
        attrs["dtype"] = _TY_DTYPE.get(op.sig.ret.name, torch.float64)
    if kind == "Cast":
        attrs["ty"] = op.sig.ret.name
    if kind in ("Reshape", "Broadcast") and len(op.inputs) == 2:
        attrs.pop("shape", None)  # the shape is the operand
    if kind == "BitDecompose":
        attrs["to_bits"] = bits == 1
    params = _params(prim.impl)
    if params is not None:  # drop IR-only attributes (e.g. scaling_base)
        attrs = {k: v for k, v in attrs.items() if k in params}
    return attrs


_PARAMS = {}


def _params(fn):
    import inspect

    p = _PARAMS.get(fn, False)
    if p is False:
        sig = inspect.signature(fn)
        if any(x.kind == x.VAR_KEYWORD for x in sig.parameters.values()):
            p = None
        else:
            p = set(sig.parameters)
        _PARAMS[fn] = p
    return p


def _cross(kind, x0, x1, y0, y1):
    if kind == "RingDotCross":
        return R.dot_cross(x0, x1, y0, y1, nb=0)
    return R.rss_cross("arith" if kind == "RingMulCross" else "bool", x0, x1, y0, y1, None, 0, 1)
