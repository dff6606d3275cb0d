"""Point-to-point value transport between party processes over ``torch.distributed``.

This replaces the reference's networking layer (``moose/src/networking``: the
``AsyncNetworking{send, receive}`` trait keyed by (SessionId, RendezvousKey), gRPC in
``networking/grpc.rs:98-170`` and TCP streams in ``networking/tcpstream.rs:160-284``).
On a MI355X node every party is one process on its own GPU and every message is an
RCCL ``send``/``recv`` over xGMI (backend ``"nccl"`` is RCCL on ROCm); CPU tests use the
``gloo`` backend with the same code.

Matching: all party processes execute the same protocol program in the same order
(SPMD), so the n-th message from A to B is always the n-th receive B posts from A --
the role the reference's rendezvous keys play.  Messages whose shape the receiver
already knows (the hot reshare path, :meth:`Transport.shift`) go without a header;
everything else is preceded by a fixed-size int64 header describing the payload
(kind, dtype, ring width, shape) so that no Python object is ever pickled.
"""
from __future__ import annotations

import collections
import math
import os
import struct
import time
from typing import List

import torch
import torch.distributed as dist

from moose_amd import errors
from moose_amd.ops import ring as R

HEADER_WORDS = 24
MAX_DIMS = HEADER_WORDS - 4

# payload kinds
K_RT, K_TENSOR, K_BYTES, K_SHAPE, K_INT, K_FLOAT, K_NONE, K_STR, K_BOOL = range(9)

_DTYPES = [torch.float64, torch.float32, torch.int64, torch.int32, torch.uint8, torch.bool,
           torch.int8, torch.int16, torch.float16, torch.bfloat16]
_DTYPE_CODE = {d: i for i, d in enumerate(_DTYPES)}


class TransportError(errors.Networking):
    pass


# Message plans (header replay).  Every party process runs the same program, so for a given
# computation and argument shapes the sequence of typed messages between two processes --
# kinds, dtypes, ring widths, shapes -- is the same in every evaluation.  The first
# evaluation under a plan key sends headers and records them on both sides; later ones
# send payloads only and take the headers from the plan, so no message makes the receiver
# read a header back to the host (the reference ships HostShape metadata with every Share,
# replicated/convert.rs:49-160).  A sender whose header differs from the plan raises
# instead of desynchronising its peer.  Least-recently-used first out, so a long-lived
# worker that sees many argument shapes keeps a bounded table.
_PLANS: "collections.OrderedDict" = collections.OrderedDict()
PLAN_CACHE = int(os.environ.get("MOOSEX_MSG_PLANS", "256"))
# send-only rounds in flight per transport before the oldest is waited for
MAX_UNWAITED = 64


class _Plan:
    __slots__ = ("inb", "outb")

    def __init__(self):
        self.inb = {}   # src rank -> [header, ...] received in order
        self.outb = {}  # dst rank -> [header, ...] sent in order


class Transport:
    """Typed send/recv between the ranks of a process group.

    ``device`` is where payload tensors travel (a CUDA device for RCCL, CPU for gloo).
    """

    def __init__(self, rank: int, world: int, device, group=None, fault=None,
                 plans: bool = False, plan_scope=None):
        self.rank = rank
        # message plans (module doc of _PLANS): only for runtimes that hand every process
        # every argument, so that all processes derive the same plan key
        self.plans = plans
        # plans are shared by the transports of one scope: a process that runs the same
        # computation under another argument layout (e.g. a party that holds no argument,
        # so its key cannot see the others' shapes) uses a scope of its own for it
        self.plan_scope = plan_scope
        self.world = world
        self.device = torch.device(device)
        self.group = group
        self.bytes_sent = 0
        self.messages = 0
        # test-only fault injection: MOOSEX_FAULT="drop:<k>@<rank>" drops this rank's
        # k-th outgoing message, "delay:<seconds>@<rank>" delays every send,
        # "exit:<k>@<rank>" kills the process at its k-th grouped exchange
        self.fault = fault if fault is not None else _parse_fault(os.environ.get("MOOSEX_FAULT"),
                                                                   rank)
        self._sends = 0
        self._mode = None  # message plan: None, "record" or "replay"
        self._plan = None
        self.header_recvs = 0  # headers read back from the device (record / no plan)
        # gloo with device tensors (CPU tests, one-GPU rehearsals of multi-rank layouts):
        # stage payloads through host memory explicitly, as parallel/cyclic.RingComm does
        try:
            backend = dist.get_backend(group) if world > 1 else "none"
        except (RuntimeError, ValueError):
            backend = "none"
        self.stage = backend == "gloo" and self.device.type == "cuda"
        # RCCL: a send-only round does not hold the compute stream (exchange); gloo only on
        # request (MOOSEX_ASYNC_SENDS=1: CPU tests of the completion checks)
        self.async_sends = backend == "nccl" or (
            backend == "gloo" and os.environ.get("MOOSEX_ASYNC_SENDS") == "1")
        self._unwaited = []  # [(work, dst)] of send-only rounds not yet known complete
        # tape mode (parallel/spmd_graphs.py): every message round is handed to this
        # callback as a CommStep instead of being sent -- the capture of a replayable
        # evaluation, where no data exists yet
        self.tape = None

    # -- encoding -----------------------------------------------------------------
    def _header(self, v):
        h = [0] * HEADER_WORDS
        payload = None
        if isinstance(v, R.RT):
            h[0], h[2] = K_RT, v.bits
            data = v.data
            payload = data
            shape = tuple(data.shape)
            h[1] = _DTYPE_CODE[data.dtype]
        elif isinstance(v, torch.Tensor):
            h[0] = K_TENSOR
            data = v
            if data.dtype == torch.bool:  # RCCL has no bool reduction type; ship bytes
                h[2] = 1
                data = data.to(torch.uint8)
            h[1] = _DTYPE_CODE[data.dtype]
            payload = data
            shape = tuple(data.shape)
        elif isinstance(v, (bytes, bytearray)):
            h[0], h[1] = K_BYTES, _DTYPE_CODE[torch.uint8]
            payload = torch.tensor(list(v), dtype=torch.uint8)
            shape = (len(v),)
        elif isinstance(v, str):
            h[0], h[1] = K_STR, _DTYPE_CODE[torch.uint8]
            b = v.encode()
            payload = torch.tensor(list(b), dtype=torch.uint8)
            shape = (len(b),)
        elif isinstance(v, bool):
            h[0], h[4] = K_BOOL, int(v)
            return h, None
        elif isinstance(v, int):
            h[0] = K_INT
            # two's-complement 128-bit split (Python ints used as ring constants)
            u = v & ((1 << 128) - 1)
            h[4], h[5] = _s64(u & ((1 << 64) - 1)), _s64(u >> 64)
            h[6] = 1 if v < 0 else 0
            return h, None
        elif isinstance(v, float):
            h[0] = K_FLOAT
            h[4] = struct.unpack("<q", struct.pack("<d", v))[0]
            return h, None
        elif v is None:
            h[0] = K_NONE
            return h, None
        elif isinstance(v, tuple) and all(isinstance(d, int) for d in v):
            h[0] = K_SHAPE
            if len(v) > MAX_DIMS:
                raise TransportError(f"shape {v} has too many dimensions")
            h[3] = len(v)
            h[4:4 + len(v)] = list(v)
            return h, None
        else:
            raise TransportError(f"cannot transport a {type(v).__name__}")
        if len(shape) > MAX_DIMS:
            raise TransportError(f"tensor of rank {len(shape)} is too large to transport")
        h[3] = len(shape)
        h[4:4 + len(shape)] = list(shape)
        return h, payload

    def _decode_header(self, h: List[int]):
        kind = h[0]
        if kind == K_BOOL:
            return kind, None, bool(h[4])
        if kind == K_INT:
            u = (h[4] & ((1 << 64) - 1)) | ((h[5] & ((1 << 64) - 1)) << 64)
            return kind, None, u - (1 << 128) if h[6] else u
        if kind == K_FLOAT:
            return kind, None, struct.unpack("<d", struct.pack("<q", h[4]))[0]
        if kind == K_NONE:
            return kind, None, None
        shape = tuple(h[4:4 + h[3]])
        if kind == K_SHAPE:
            return kind, None, shape
        return kind, shape, None

    # -- raw tensors ----------------------------------------------------------------
    def _send_tensor(self, t: torch.Tensor, dst: int):
        t = t.contiguous()
        if t.device != self.device:
            t = t.to(self.device)
        if t.numel() == 0:
            return
        self._sends += 1
        if self.fault is not None:
            kind, val = self.fault
            if kind == "drop" and self._sends == val:
                return  # the receiver waits until the session deadline
            if kind == "delay":
                time.sleep(val)
        dist.send(t.cpu() if self.stage else t, dst, group=self.group)
        self.bytes_sent += t.numel() * t.element_size()
        self.messages += 1

    def _recv_tensor(self, shape, dtype, src: int) -> torch.Tensor:
        t = torch.empty(shape, dtype=dtype, device="cpu" if self.stage else self.device)
        if t.numel() == 0:
            return t.to(self.device)
        dist.recv(t, src, group=self.group)
        return t.to(self.device) if self.stage else t

    # -- message plans ----------------------------------------------------------------
    def begin_plan(self, key):
        """Start an evaluation under plan ``key`` (identical on every process): replay the
        recorded headers if the plan exists, else record them."""
        p = _PLANS.get((self.plan_scope, self.rank, self.world, key))
        if p is not None:
            _PLANS.move_to_end((self.plan_scope, self.rank, self.world, key))
        self._plan_key = key
        self._cursor_in, self._cursor_out = {}, {}
        if p is not None:
            self._mode, self._plan = "replay", p
        else:
            self._mode, self._plan = "record", _Plan()

    def end_plan(self, ok: bool = True):
        if self._mode == "record" and ok:
            _PLANS[(self.plan_scope, self.rank, self.world, self._plan_key)] = self._plan
            while len(_PLANS) > PLAN_CACHE:
                _PLANS.popitem(last=False)
        self._mode = self._plan = None

    # -- completion of send-only rounds ------------------------------------------------
    def _failed(self, w, dst, err):
        self._unwaited = []
        raise TransportError(f"rank {self.rank}: send to rank {dst} failed: {err}")

    def reap(self, block: bool = False):
        """Observe the send-only rounds still in flight: a completed one that failed raises
        :class:`TransportError` here, on the SENDER (not only as a timeout on its peer);
        ``block`` waits for all of them (end of an evaluation)."""
        keep = []
        for w, dst in self._unwaited:
            # a completed work's wait() returns at once or raises its error (gloo reports a
            # dead peer only through wait(); Work.exception() is not usable from Python)
            if block or w.is_completed():
                try:
                    w.wait()
                except Exception as e:  # noqa: BLE001 - any backend error
                    self._failed(w, dst, e)
            else:
                keep.append((w, dst))
        self._unwaited = keep

    def end_evaluation(self):
        """Every send of the evaluation confirmed (or its failure raised)."""
        if self.tape is None:
            self.reap(block=True)

    def _next(self, cursors, peer):
        k = cursors.get(peer, 0)
        cursors[peer] = k + 1
        return k

    # -- tape mode ----------------------------------------------------------------------
    def _taped(self, sends, recvs):
        """Tape mode: hand the round to the tape (parallel/spmd_graphs.py).  Sends are
        made contiguous first (inside the capture, so the copy is replayed); receives land
        in contiguous buffers whose copy into ``out`` is captured after the round."""
        sends = [(t.contiguous(), dst) for t, dst in sends if t.numel()]
        land, after = [], []
        for out, src in recvs:
            if out.numel() == 0:
                continue
            if out.is_contiguous():
                land.append((out, src))
            else:
                buf = torch.empty(out.shape, dtype=out.dtype, device=out.device)
                land.append((buf, src))
                after.append((out, buf))
        self.tape(CommStep(sends, land))
        for out, buf in after:  # captured in the segment after the round
            out.copy_(buf)

    # -- typed values -----------------------------------------------------------------
    def send(self, v, dst: int):
        h, payload = self._header(v)
        if self._mode == "replay":
            rec = self._plan.outb.get(dst, [])
            k = self._next(self._cursor_out, dst)
            if k >= len(rec) or rec[k] != h:
                raise TransportError(
                    f"message {k} to rank {dst} does not match the evaluation's message plan "
                    "(data-dependent shapes?)")
        else:
            self._send_tensor(torch.tensor(h, dtype=torch.int64), dst)
            if self._mode == "record":
                self._plan.outb.setdefault(dst, []).append(h)
        if payload is not None:
            if self.tape is not None:
                if self._mode != "replay":
                    raise TransportError("tape mode needs a recorded message plan")
                self._taped([(payload.to(self.device), dst)], [])
                return
            self._send_tensor(payload, dst)

    def recv(self, src: int, device=None):
        if self._mode == "replay":
            rec = self._plan.inb.get(src, [])
            k = self._next(self._cursor_in, src)
            if k >= len(rec):
                raise TransportError(f"message {k} from rank {src} is not in the message plan")
            h = rec[k]
        else:
            h = self._recv_tensor((HEADER_WORDS,), torch.int64, src).cpu().tolist()
            self.header_recvs += 1
            if self._mode == "record":
                self._plan.inb.setdefault(src, []).append(h)
        kind, shape, scalar = self._decode_header(h)
        if shape is None:
            return scalar
        dtype = _DTYPES[h[1]]
        if self.tape is not None:
            if kind in (K_BYTES, K_STR):
                raise TransportError("tape mode: a host value (bytes) in the message flow")
            data = torch.empty(shape, dtype=dtype, device=self.device)
            self._taped([], [(data, src)])
        else:
            data = self._recv_tensor(shape, dtype, src)
        if device is not None:
            data = data.to(device)
        if kind == K_RT:
            return R.RT(data, h[2])
        if kind == K_TENSOR:
            return data.to(torch.bool) if h[2] == 1 else data
        if kind == K_BYTES:
            return bytes(data.cpu().tolist())
        if kind == K_STR:
            return bytes(data.cpu().tolist()).decode()
        raise TransportError(f"bad header kind {kind}")

    # -- structured exchanges ------------------------------------------------------------
    def shift(self, t: torch.Tensor, to_rank: int, from_rank: int) -> torch.Tensor:
        """Send ``t`` to ``to_rank`` while receiving a same-shaped tensor from
        ``from_rank`` (the RSS reshare ring).  One grouped RCCL call."""
        t = t.contiguous()
        if t.device != self.device:
            t = t.to(self.device)
        out = torch.empty_like(t)
        if t.numel() == 0:
            return out
        if self.tape is not None:
            self._taped([(t, to_rank)], [(out, from_rank)])
            return out
        st, so = (t.cpu(), torch.empty(t.shape, dtype=t.dtype)) if self.stage else (t, out)
        ops = [dist.P2POp(dist.isend, st, to_rank, group=self.group),
               dist.P2POp(dist.irecv, so, from_rank, group=self.group)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        if self.stage:
            out.copy_(so)
        self.bytes_sent += t.numel() * t.element_size()
        self.messages += 1
        return out

    def exchange(self, sends, recvs):
        """One grouped round of header-free point-to-point messages: ``sends`` is a list of
        (tensor, dst), ``recvs`` a list of (preallocated tensor, src) whose shapes both
        sides know (protocol messages of a known element count)."""
        if self.tape is not None:
            self._taped(sends, recvs)
            return
        ops, staged = [], []
        for t, dst in sends:
            t = t.contiguous()
            if t.numel() == 0:
                continue
            ops.append(dist.P2POp(dist.isend, t.cpu() if self.stage else t, dst,
                                  group=self.group))
            self.bytes_sent += t.numel() * t.element_size()
            self.messages += 1
        for out, src in recvs:
            if out.numel() == 0:
                continue
            if self.stage or not out.is_contiguous():
                # a contiguous landing buffer (host memory when staging), copied into out
                buf = torch.empty(out.shape, dtype=out.dtype,
                                  device="cpu" if self.stage else out.device)
                staged.append((out, buf))
            else:
                buf = out
            ops.append(dist.P2POp(dist.irecv, buf, src, group=self.group))
        if self._unwaited:
            self.reap()  # a failed earlier send surfaces at the sender's next round
        if self.fault is not None and self.fault[0] == "delay":
            time.sleep(self.fault[1])  # test-only: this rank joins every round late
        if self.fault is not None and self.fault[0] == "exit":
            self._sends += 1
            if self._sends == self.fault[1]:
                os._exit(17)  # test-only: this rank dies before its k-th round (a lost peer)
        if ops:
            works = dist.batch_isend_irecv(ops)
            if recvs or not self.async_sends:
                for w in works:
                    w.wait()
            else:
                # a send-only round (a share's owner, the dealer, the revealing party): the
                # compute stream goes on while the bytes travel -- nothing here reads what
                # a send delivers, and the process group keeps the payload alive until the
                # transfer is done (its RCCL stream runs the round's messages in order).
                # Completion is observed at the next rounds and at the evaluation's end.
                dst = sends[0][1] if sends else -1
                self._unwaited.extend((w, dst) for w in works)
                while len(self._unwaited) > MAX_UNWAITED:  # bound: wait for the oldest
                    w, d = self._unwaited.pop(0)
                    try:
                        w.wait()
                    except Exception as e:  # noqa: BLE001
                        self._failed(w, d, e)
        for out, buf in staged:
            out.copy_(buf)

    def broadcast_from(self, v, src: int, dsts: List[int], me: int):
        """``src`` sends ``v`` to every rank in ``dsts``; returns the value at ``me``."""
        if me == src:
            for d in dsts:
                if d != src:
                    self.send(v, d)
            return v
        if me in dsts:
            return self.recv(src)
        return None


class CommStep:
    """One message round of a taped evaluation (parallel/spmd_graphs.py): the round's
    sends and receives with the device buffers they were recorded with, re-issued as one
    grouped, header-free exchange at every replay."""

    __slots__ = ("sends", "recvs")

    def __init__(self, sends, recvs):
        self.sends = sends
        self.recvs = recvs

    def run(self, tr: "Transport"):
        tr.exchange(self.sends, self.recvs)


def _parse_fault(spec, rank):
    if not spec:
        return None
    if spec == "party_landing":  # parallel/threads.py: per-party stream graphs only
        return None
    what, _, who = spec.partition("@")
    if who and int(who) != rank:
        return None
    kind, _, val = what.partition(":")
    if kind == "drop":
        return ("drop", int(val))
    if kind == "delay":
        return ("delay", float(val))
    if kind == "exit":  # the process dies at its k-th grouped exchange (a lost peer)
        return ("exit", int(val))
    raise ValueError(f"bad MOOSEX_FAULT spec {spec!r}")


def _s64(u: int) -> int:
    return u - (1 << 64) if u >= (1 << 63) else u


def payload_bytes(v) -> int:
    if isinstance(v, R.RT):
        if v.bits in (64, 128):  # without touching data (lazy Encoded / Opened)
            return v.numel() * (v.bits // 8)
        return v.data.numel() * v.data.element_size()
    if isinstance(v, torch.Tensor):
        return v.numel() * v.element_size()
    if isinstance(v, (bytes, bytearray, str)):
        return len(v)
    return 8


def numel(shape) -> int:
    return int(math.prod(shape)) if shape else 1


__all__ = ["Transport", "TransportError", "CommStep", "payload_bytes", "numel"]
