"""Native dataflow execution of lowered (host-only) computations.

Parity: reference ``execution/asynchronous.rs`` -- ``AsyncSession`` turns every
operation into a task that runs once its operands are ready (:477-528), Send/Receive go
through ``AsyncNetworking`` keyed by rendezvous key (:240-317), ``AsyncExecutor`` runs
only the operations its identity owns (:579-605), and the first root-cause error aborts
the session (``join_on_first_error`` :32-73).  ``networking/tcpstream.rs`` is the raw-TCP
backend (one stream per peer, length-prefixed frames).

Here the scheduler is the C++ ``Dataflow`` of ``csrc/runtime/scheduler.cpp``: it tracks
readiness from the native ``Graph``, parks a Receive until its rendezvous key has
arrived in the native ``Mailbox`` (so a worker thread never blocks on the network), and
calls back into Python only to run the operation's kernel.  Two networking modes:

* in-process (``identity=None``): every identity in one process; a Send parks the value
  and posts its key to the mailbox, the Receive picks it up (``LocalAsyncNetworking``);
* per identity over TCP (:class:`TcpTransport`): the native ``TcpNetworking`` moves typed
  frames (int64 header + raw tensor bytes, no pickling) between identity processes on
  any hosts -- the cross-node path; intra-node GPU runs use RCCL (``parallel/``).
"""
from __future__ import annotations

import os
import struct
from typing import Dict
from typing import Optional

import numpy as np
import torch

from moose_amd.ops import ring as R
from moose_amd.parallel import transport as PT
from moose_amd.runtime import native_rt as N


def tls_files(identity: str, certs_dir: str):
    """``{certs_dir}/{identity}.crt``, ``{identity}.key`` and ``ca.crt`` -- the layout of
    the reference's ``load_identity_and_ca`` (reindeer.rs:65-78).  The certificate's
    common name must be the identity."""
    files = (os.path.join(certs_dir, f"{identity}.crt"), os.path.join(certs_dir, f"{identity}.key"),
             os.path.join(certs_dir, "ca.crt"))
    for f in files:
        if not os.path.exists(f):
            raise FileNotFoundError(f"TLS file missing: {f}")
    return files


class TcpTransport:
    """Typed value transport between identity processes over the native TCP networking.

    ``endpoints``: identity -> "host:port" for every identity (own entry = listen address;
    port 0 picks a free one, see :attr:`port`).  ``certs_dir``: mutual TLS with the
    certificates of :func:`tls_files`; peers are authenticated by certificate CN.
    """

    def __init__(self, identity: str, endpoints: Dict[str, str], session_id: str = "",
                 connect_timeout_s: float = 300.0, certs_dir: Optional[str] = None):
        m = N.mod()
        self.identity = identity
        self.session_id = session_id
        self.mailbox = m.Mailbox()
        tls = tls_files(identity, certs_dir) if certs_dir else ("", "", "")
        self.net = m.TcpNetworking(identity, dict(endpoints), self.mailbox,
                                   max_elapsed_s=connect_timeout_s, cert_file=tls[0],
                                   key_file=tls[1], ca_file=tls[2])
        self._codec = PT.Transport(0, 1, "cpu")  # header encoder only
        self.started = False

    def start(self):
        if not self.started:
            self.net.start()
            self.started = True
        return self

    @property
    def port(self) -> int:
        return self.net.port

    def key(self, rdv_hex: str) -> str:
        return f"{self.session_id}/{rdv_hex}"

    # -- codec ---------------------------------------------------------------------
    def encode(self, v) -> bytes:
        h, payload = self._codec._header(v)
        head = struct.pack(f"<{PT.HEADER_WORDS}q", *h)
        if payload is None:
            return head
        t = payload.detach().contiguous().cpu()
        return head + t.view(torch.uint8).numpy().tobytes() if t.numel() else head

    def decode(self, data: bytes, device):
        hw = PT.HEADER_WORDS * 8
        h = list(struct.unpack(f"<{PT.HEADER_WORDS}q", data[:hw]))
        kind, shape, scalar = self._codec._decode_header(h)
        if shape is None:
            return scalar
        dtype = PT._DTYPES[h[1]]
        buf = np.frombuffer(data, dtype=np.uint8, offset=hw).copy()
        t = torch.from_numpy(buf).view(dtype).reshape(shape) if buf.size else \
            torch.empty(shape, dtype=dtype)
        t = t.to(device)
        if kind == PT.K_RT:
            return R.RT(t, h[2])
        if kind == PT.K_TENSOR:
            return t.to(torch.bool) if h[2] == 1 else t
        if kind == PT.K_BYTES:
            return bytes(t.cpu().numpy().tobytes())
        if kind == PT.K_STR:
            return bytes(t.cpu().numpy().tobytes()).decode()
        raise PT.TransportError(f"bad header kind {kind}")

    # -- messaging -------------------------------------------------------------------
    def send_value(self, receiver: str, rdv_hex: str, v):
        self.net.send(receiver, self.key(rdv_hex), self.encode(v))

    def take_value(self, rdv_hex: str, device, timeout_s: float = 0.0):
        _, payload = self.mailbox.take(self.key(rdv_hex), timeout_s)
        return self.decode(payload, device)

    def flush(self, timeout_s: float = 300.0):
        self.net.flush(timeout_s)

    def stats(self):
        return self.net.stats()

    def close(self):
        self.net.close()


def default_workers() -> int:
    return int(os.environ.get("MOOSEX_DATAFLOW_WORKERS", "1"))


def run_dataflow(executor, comp, arguments: Optional[dict], workers: Optional[int] = None,
                 timeout_s: float = -1.0) -> dict:
    """Run ``comp`` on ``executor`` (a :class:`GraphExecutor`) with the native scheduler.

    ``executor.identity`` None: all identities in this process.  Otherwise only that
    identity's operations run and ``executor.tr`` must be a :class:`TcpTransport`.
    """
    from moose_amd.runtime.graph_executor import GraphExecutionError
    from moose_amd.runtime.interpreter import numpy_to_torch

    m = N.mod()
    arguments = arguments or {}
    ops = comp.operations
    try:
        g = N.graph_of(comp)
    except m.NativeGraphError as e:
        msg = str(e)
        if "two Send" in msg:
            raise GraphExecutionError(f"duplicate send: {msg}") from None
        raise GraphExecutionError(msg) from None
    me = executor.identity
    tr = executor.tr
    local = me is None
    mb = m.Mailbox() if local else tr.mailbox
    sends = {N.rdv_hex(op) for op in ops if op.kind == "Send"}
    mine, keys = [], []
    for i, op in enumerate(ops):
        if not local and op.placement.owner != me:
            continue
        mine.append(i)
        if op.kind == "Receive":
            k = N.rdv_hex(op)
            if local and k not in sends:
                raise GraphExecutionError(f"receive {op.name}: no Send for its rendezvous key")
            keys.append(k if local else tr.key(k))
        else:
            keys.append("")
    env: Dict[str, object] = {}
    parked: Dict[str, object] = {}
    outputs: dict = {}
    executor._used = set()
    device = executor.device

    def step(i):
        op = ops[i]
        kind = op.kind
        if kind == "Send":
            k = N.rdv_hex(op)
            v = env[op.inputs[0]]
            if local:
                parked[k] = v
                mb.put(k, op.placement.owner, b"")
            else:
                tr.send_value(op.attrs["receiver"], k, v)
            return
        if kind == "Receive":
            k = N.rdv_hex(op)
            if local:
                mb.take(k, 0.0)
                env[op.name] = parked.pop(k)
            else:
                env[op.name] = tr.take_value(k, device)
            return
        try:
            env[op.name] = executor._exec(op, env, parked, arguments, outputs, {}, numpy_to_torch)
        except GraphExecutionError:
            raise
        except Exception as e:
            raise GraphExecutionError(
                f"{op.name} = {kind} @ {op.placement.owner} failed: {e}") from e

    df = m.Dataflow(g, mine, keys, mb)
    try:
        executor.last_run_stats = df.run(step, workers or default_workers(), timeout_s)
    except m.NativeNetError as e:
        raise GraphExecutionError(str(e)) from None
    if not local:
        tr.flush()
    return outputs
