"""Cyclic multi-GPU layout: N concurrent 3-party sessions on N GPUs, every party of a
session on its own GPU, every reshare an RCCL send/recv over xGMI.

Placement rule: role ``r`` (offset ``o(r)``: 0, 1, 2 for the three parties of the
replicated placement -- 0, 1, 3 on >= 4 GPUs, so that every inter-party flow gets its own
xGMI link (:func:`default_offsets`) -- further roles after them) of session ``s`` lives on GPU
``(s + o(r)) mod N``.  So GPU ``g`` hosts role ``r`` of session ``(g - o(r)) mod N`` --
one instance of EVERY role, each from a different session (for N >= 3):

    N = 4      GPU0          GPU1          GPU2          GPU3
    alice      s0            s1            s2            s3
    bob        s3            s0            s1            s2
    carole     s2            s3            s0            s1

Every GPU therefore does exactly the work of one stacked 3-party session (the weak-scaling
unit of the 1-GPU bench), with the SAME batched kernels: a party vector is still one
``[3, ...]`` tensor whose component ``p`` is party ``p`` -- of session ``g - o(owner_p)``.
What changes is data movement, which becomes real inter-GPU traffic:

* ``shift`` (the RSS reshare, component p <- component p+k of the same session) sends
  each component to the GPU holding its destination party and receives from the GPU
  holding its source party: one grouped ``batch_isend_irecv``, zero-copy into the
  component slices;
* ``move`` of a host value from role a to role b is a ring shift by ``o(b) - o(a)``;
* ``take``/``gather`` stay local (component p and role ``owner_p`` belong to the same
  session on this GPU).

Because all N sessions run the same program on tensors of the same shapes (data-parallel
replicas), every receiver knows the shape and dtype of what it receives from its own
local copy: transfers carry no header and never synchronise with the host.  Public
(mirrored) values are assumed replica-invariant (e.g. model weights); secret inputs may
differ per session.

Correlated randomness: each component has its OWN key pair (k_p, k_{p+1}) and k_all of
its session -- the three components of a stack belong to different sessions, so the
stacked zero-share kernels run in "pairs" mode (``mx_rss_cross_kp``).  Key setup follows
``replicated/setup.rs:39-58``: party p draws k_p and hands a copy to party p-1 (here: its
device key slot -- the raw 128-bit ChaCha12 key -- sent device to device); party 0 draws
k_all and passes it on.

With N = 1 the layout degenerates to one stacked session (every offset is 0 mod 1), which
is what ``bench.py`` runs on one GPU (with the fully fused single-GPU kernels).

Reference parity: the reference runs each party as its own worker process exchanging
bincode values over gRPC (``execution/asynchronous.rs:557-632``, ``networking/grpc.rs``);
its benchmark reports the max over the three workers (``benchmarks/pymoose/
dot_product.py:124-139``).  This layout is that deployment, replicated N times across a
node so that all N GPUs are busy.
"""
from __future__ import annotations

import hashlib
import os
from typing import Dict
from typing import List
from typing import Sequence
from typing import Tuple

import torch
import torch.distributed as dist

from moose_amd.ops import ring as R
from moose_amd.runtime.session import HV
from moose_amd.runtime.session import PV
from moose_amd.runtime.session import StackedSession
from moose_amd.runtime.session import _nbytes


class RingComm:
    """Header-free symmetric point-to-point exchange over a process group.

    ``exchange(sends, recvs)``: ``sends`` = [(tensor, dst_rank)], ``recvs`` =
    [(out_tensor, src_rank)].  Every rank calls it with mirror-image lists (the n-th send
    from A to B pairs with the n-th receive at B from A).  On RCCL the transfers are one
    grouped ``batch_isend_irecv`` whose completion is a stream dependency, never a host
    wait; transfers to oneself are device copies.  On gloo with device tensors the
    payloads are staged through host memory (CPU tests and the one-GPU rehearsal).
    """

    def __init__(self, rank: int, world: int, device, group=None):
        self.rank = rank
        self.world = world
        self.device = torch.device(device)
        self.group = group
        backend = dist.get_backend(group) if world > 1 else "none"
        self.stage = backend == "gloo" and self.device.type == "cuda"
        self.bytes_sent = 0
        self.messages = 0
        self.rounds = 0

    def exchange(self, sends: Sequence[Tuple[torch.Tensor, int]],
                 recvs: Sequence[Tuple[torch.Tensor, int]]):
        local_s = [t for t, r in sends if r == self.rank]
        local_r = [t for t, r in recvs if r == self.rank]
        if len(local_s) != len(local_r):
            raise RuntimeError("unbalanced self-exchange")
        for src, out in zip(local_s, local_r):
            out.copy_(src)
        ops = []
        staged = []
        for t, r in sends:
            if r == self.rank or t.numel() == 0:
                continue
            t = t.contiguous()
            if self.stage:
                t = t.cpu()
            ops.append(dist.P2POp(dist.isend, t, r, group=self.group))
            self.bytes_sent += t.numel() * t.element_size()
            self.messages += 1
        for out, r in recvs:
            if r == self.rank or out.numel() == 0:
                continue
            if self.stage:
                # pinned: the copy into ``out`` below is asynchronous, and the host caching
                # allocator keeps a pinned buffer alive until that copy has run (a pageable
                # buffer could be freed and reused while the DMA still reads it)
                buf = torch.empty(out.shape, dtype=out.dtype, pin_memory=True)
                staged.append((out, buf))
                ops.append(dist.P2POp(dist.irecv, buf, r, group=self.group))
            else:
                ops.append(dist.P2POp(dist.irecv, out, r, group=self.group))
        if not ops:
            return
        self.rounds += 1
        for w in dist.batch_isend_irecv(ops):
            w.wait()  # RCCL: the current stream waits; gloo: completes the transfer
        for out, buf in staged:
            out.copy_(buf, non_blocking=True)


def dot_traffic(dirs=(1, 1)):
    """Per-step traffic between the three parties of one session of the dot-product program
    (x owned by party 0, y by party 1, output revealed to party 2), in units of one share
    tensor of the output: the input shares (owner j -> P_{j+d}, d = its share direction)
    and the folded dot tail with the reveal merged into its last round (parallel/party.py:
    m0 0->1; m1 1->0; z2 2->0 and 2->1; rt1, rm1 2->1; w0 0->2, w1 1->2)."""
    f = {(0, 1): 1.0, (1, 0): 1.0, (2, 0): 1.0, (2, 1): 2.5, (0, 2): 1.0, (1, 2): 1.0}
    for owner, d in ((0, dirs[0]), (1, dirs[1])):
        key = (owner, (owner + d) % 3)
        f[key] = f.get(key, 0.0) + 1.0
    return f


TRAFFIC = dot_traffic()


def link_loads(offsets: Sequence[int], world: int, traffic=None) -> Dict[int, float]:
    """Per-GPU traffic on each outgoing link ``g -> g + d`` (key ``d``), for party offsets
    ``offsets``.  Every GPU runs the same pattern, so link ``d`` of every GPU carries the sum
    of the flows whose offset difference is ``d`` mod ``world``; ``d = 0`` is a local copy."""
    load: Dict[int, float] = {}
    for (a, b), w in (traffic or TRAFFIC).items():
        d = (offsets[b] - offsets[a]) % world
        load[d] = load.get(d, 0.0) + w
    return load


def default_layout(roles: Sequence[str], world: int = None):
    """(offsets, share directions) of the roles for the dot-product program on ``world``
    GPUs: the pair minimising the busiest link (:func:`dot_traffic`, :func:`link_loads`);
    ties keep the reference's share direction.  E.g. 8 GPUs: offsets (0, 1, 3), every flow
    on its own link, the busiest one 2.5 units (4.5 with offsets 0, 1, 2); 4 GPUs: offsets
    (0, 2, 1), 3.5 units.  The mirrored share direction wins for other traffic patterns
    (before the reveal was merged into the tail, it took 8 GPUs from 3 units to 2.5)."""
    n = len(roles)
    off = default_offsets(roles, world)
    if world is None or world < 4 or n < 3:
        return off, {}
    best = None
    for dx in (1, 2):
        for dy in (1, 2):
            fl = dot_traffic((dx, dy))
            for o1 in range(1, world):
                for o2 in range(1, world):
                    if o1 == o2:
                        continue
                    o = (0, o1, o2)
                    key = (max(link_loads(o, world, fl).values()), (dx, dy) != (1, 1), dx, dy, o)
                    if best is None or key < best[0]:
                        best = (key, o, dx, dy)
    _, o, dx, dy = best
    rest = [k for k in range(max(world, n)) if k not in o]
    offsets = {r: v for r, v in zip(roles, list(o) + rest[:n - 3])}
    dirs = {r: d for r, d in ((roles[0], dx), (roles[1], dy)) if d != 1}
    return offsets, dirs


def default_offsets(roles: Sequence[str], world: int = None) -> Dict[str, int]:
    """Offsets of the roles (module doc): 0, 1, 2, ... unless ``world`` GPUs allow a
    link-balanced choice (for the reference's share direction; :func:`default_layout`
    chooses the share directions too).

    xGMI is point to point -- every GPU pair has its own link (≈50-64 GB/s per direction
    under RCCL) -- so the step time of a communication-heavy program is set by the busiest
    link, not the total volume.  With offsets (0, 1, 2) several flows of the dot program
    share a distance (4.5 of its 9.5 units on one link on 8 GPUs); for ``world >= 4`` the
    offsets of the three parties are chosen to minimise the busiest link, e.g. (0, 1, 3) on
    8 GPUs puts every flow on its own link (2.5 units).
    Further roles take the smallest unused offsets."""
    n = len(roles)
    off = list(range(n))
    if world is not None and world >= 4 and n >= 3:
        cands = [(0, o1, o2) for o1 in range(1, world) for o2 in range(1, world) if o1 != o2]
        best = min(cands, key=lambda o: (max(link_loads(o, world).values()), o))
        rest = [k for k in range(max(world, n)) if k not in best]
        off = list(best) + rest[:n - 3]
    return {r: o for r, o in zip(roles, off)}


# MOOSEX_DEALER_SIDE=1: the dot tail's early dealer kernel on a side stream beside the GEMM
# (one GPU).  Off: measured slower -- 16.68 -> 16.90-16.99 ms per cyclic step on one MI355X
# (gpurun_out/r5v): the ChaCha kernel next to the power-bound GEMM costs it more clock than
# it hides
DEALER_SIDE = os.environ.get("MOOSEX_DEALER_SIDE", "0") == "1"


class CyclicSession(StackedSession):
    """Stacked party vectors whose components belong to N different sessions (module
    doc).  Runs the generic (per-round) protocol code; every round's messages are one
    grouped exchange."""

    is_simulated = False
    fused = False      # the single-GPU whole-protocol kernels assume all parties local
    ks_fused = False
    pair_rolled = False  # component p + 1 of a stack is another session's party
    KEY_SLOTS = 9      # per placement: for each component p: k_p, k_{p+1}, k_all

    def __init__(self, comm: RingComm, offsets: Dict[str, int], device="cpu", seed=None,
                 pipeline_chunks=None, share_dirs=None):
        super().__init__(device, seed)
        if share_dirs:
            self.share_dirs = dict(share_dirs)
        self.comm = comm
        if pipeline_chunks is None:
            # row-chunked dot pipeline (rep.dot_trunc): off by default -- chunking re-reads
            # the prepared B operand per chunk (GEMM 12.0 -> 15.4 ms at 8 chunks); bench.py
            # hides the exchanges behind the NEXT step's GEMM instead (two step streams with
            # one RCCL communicator each)
            pipeline_chunks = int(os.environ.get("MOOSEX_PIPELINE_CHUNKS", "1"))
        self.pipeline_chunks = pipeline_chunks
        self.g = comm.rank
        self.N = comm.world
        self.off = dict(offsets)
        if seed is not None:  # distinct per-rank stream for fresh seeds
            self._rng = torch.Generator().manual_seed(seed * 7919 + self.g)

    # -- layout helpers -------------------------------------------------------------
    def offset(self, role: str) -> int:
        try:
            return self.off[role]
        except KeyError:
            raise KeyError(f"role {role!r} has no offset in the cyclic layout") from None

    def session_of(self, role: str) -> int:
        """Index of the session whose ``role`` this GPU hosts."""
        return (self.g - self.offset(role)) % self.N

    def _peer(self, d: int) -> int:
        return (self.g + d) % self.N

    def _shift_tensor(self, plc, data: torch.Tensor, k: int) -> torch.Tensor:
        """Component q <- component (q + k) % 3 of the same session, for a stacked
        ``[3, ...]`` tensor of placement ``plc`` (grouped exchange, zero-copy slices)."""
        data = data.contiguous()
        out = torch.empty_like(data)
        o = [self.offset(r) for r in plc.owners]
        sends, recvs = [], []
        for q in range(3):  # iterate by DESTINATION component on both sides
            p = (q + k) % 3
            recvs.append((out[q], self._peer(o[p] - o[q])))
            sends.append((data[p], self._peer(o[q] - o[p])))
        self.comm.exchange(sends, recvs)
        return out

    # -- data movement ----------------------------------------------------------------
    def shift(self, x, k=1):
        self.stats.record_round(_nbytes(x.v))
        v = x.v
        if isinstance(v, R.RT):
            return PV(x.plc, R.RT(self._shift_tensor(x.plc, v.data, k), v.bits))
        if v.dtype == torch.bool:
            return PV(x.plc, self._shift_tensor(x.plc, v.to(torch.uint8), k).to(torch.bool))
        return PV(x.plc, self._shift_tensor(x.plc, v, k))

    def move(self, x, host):
        if x.host == host:
            return x
        d = self.offset(host) - self.offset(x.host)
        self.stats.record_send(x.host, host, _nbytes(x.v))
        if d % self.N == 0:  # both roles of that session live on this GPU
            return HV(host, x.v)
        return HV(host, self._move_value(x.v, d))

    def _move_value(self, v, d):
        dst, src = self._peer(d), self._peer(-d)
        if isinstance(v, R.RT):
            out = torch.empty_like(v.data)
            self.comm.exchange([(v.data, dst)], [(out, src)])
            return R.RT(out, v.bits)
        if isinstance(v, torch.Tensor):
            t = v.to(torch.uint8) if v.dtype == torch.bool else v
            out = torch.empty_like(t)
            self.comm.exchange([(t, dst)], [(out, src)])
            return out.to(torch.bool) if v.dtype == torch.bool else out
        if type(v).__name__ == "KeyRef":  # a fresh seed: ship its key slot (raw + schedule)
            from moose_amd.runtime.keys import KeyRef

            kt = self.keytable
            slot = kt.alloc(1)
            self.comm.exchange([(v.table.t[v.slot], dst)], [(kt.t[slot], src)])
            return KeyRef(kt, slot)
        if isinstance(v, (bytes, bytearray)):
            t = torch.tensor(list(v), dtype=torch.uint8, device=self.device)
            out = torch.empty_like(t)
            self.comm.exchange([(t, dst)], [(out, src)])
            return bytes(out.cpu().tolist())
        # shapes, Python scalars, strings: identical in every session (same program)
        return v

    def gather(self, plc, xs):
        xs = [x if x.host == plc.owners[i] else self.move(x, plc.owners[i])
              for i, x in enumerate(xs)]
        vs = [x.v for x in xs]
        if isinstance(vs[0], R.RT):
            return PV(plc, R.RT(torch.stack([v.data for v in vs]), vs[0].bits))
        return PV(plc, torch.stack(vs))

    # -- keys -------------------------------------------------------------------------
    def _seeded_key(self, plc, session: int, what) -> bytes:
        h = hashlib.blake2b(repr((self.seed, tuple(plc.owners), session, what)).encode(),
                            digest_size=16)
        return h.digest()

    def session_keys(self, plc, session: int):
        """(k_0, k_1, k_2, k_all) of ``session`` in seeded mode (tests)."""
        return [self._seeded_key(plc, session, i) for i in range(3)] + [
            self._seeded_key(plc, session, "all")]

    def setup(self, plc) -> int:
        base = self._keys.get(plc)
        if base is not None:
            return base
        kt = self.keytable
        base = kt.alloc(self.KEY_SLOTS)  # random keys everywhere
        self._keys[plc] = base
        o = [self.offset(r) for r in plc.owners]
        if self.seed is not None:
            for p in range(3):
                s = (self.g - o[p]) % self.N
                kt._write(base + 3 * p, [self._seeded_key(plc, s, p)])
                if p == 0:
                    kt._write(base + 2, [self._seeded_key(plc, s, "all")])
        # k_{p+1}: party p+1 of the same session hands a copy of its own key to party p
        own = kt.t[[base, base + 3, base + 6]]
        nxt = self._shift_tensor(plc, own, 1)
        for p in range(3):
            kt.t[base + 3 * p + 1].copy_(nxt[p])
        # k_all: drawn by party 0, passed 0 -> 1 -> 2
        kall = kt.t[[base + 2, base + 5, base + 8]]
        a = self._shift_tensor(plc, kall, 2)   # component 1 <- component 0
        b = self._shift_tensor(plc, a, 2)      # component 2 <- component 1's copy
        kt.t[base + 5].copy_(a[1])
        kt.t[base + 8].copy_(b[2])
        return base

    def _slot(self, plc, p: int, which: int) -> int:
        return self.keytable.ptr(self.setup(plc) + 3 * p + which)

    def _pair_ptrs(self, plc) -> List[int]:
        return [self._slot(plc, p, w) for p in range(3) for w in (0, 1)]

    def h_prf(self, plc, host, key_id, shape: HV, bits, nonce):
        i = plc.owners.index(host)
        if key_id == "all":
            w = 2
        elif key_id == i:
            w = 0
        elif key_id == (i + 1) % 3:
            w = 1
        else:
            raise RuntimeError(f"{host} does not hold PRF key {key_id}")
        out = R.prf_expand_k(self._slot(plc, i, w), 1, nonce, tuple(shape.v), bits, self.device)
        return HV(host, R.RT(out.data[0], bits))

    # -- RSS kernels with per-component key pairs --------------------------------------
    def p_cross(self, kind, plc, x0, x1, y0, y1, zero_share=True):
        x1v = x1.v if x1 is not None else None
        y1v = y1.v if y1 is not None else None
        nonce = self.nonce(plc)
        if not zero_share:
            return PV(plc, R.rss_cross(kind, x0.v, x1v, y0.v, y1v, None, nonce, 3))
        return PV(plc, R.rss_cross_kp(kind, x0.v, x1v, y0.v, y1v, self._pair_ptrs(plc), nonce))

    def p_cross_plain(self, kind, plc, x0, x1, y0, y1):
        """The components' cross terms with no zero share and no nonce drawn (the per-party
        tail adds the zero share)."""
        return PV(plc, R.rss_cross(kind, x0.v, x1.v, y0.v, y1.v, None, 0, 3))

    def p_add_zero_share(self, plc, z, kind="arith"):
        return PV(plc, R.rss_cross_kp(kind, z.v, None, None, None, self._pair_ptrs(plc),
                                      self.nonce(plc)))

    # -- per-party protocol rounds (csrc/rss_party.hip) ----------------------------------
    def party_trunc(self, x, m, nonces):
        """TruncPr as two per-party kernels + two grouped exchanges (+ one add): component p
        runs party p's local work of each round (replicated.trunc_pr, generic path), and
        every message goes straight to the GPU of its destination party."""
        plc, bits = x.plc, x.bits
        roles = [0, 1, 2]
        slots = self._pair_ptrs(plc)
        o = [self.offset(r) for r in plc.owners]
        p01, p10, p21 = self._peer(o[1] - o[0]), self._peer(o[0] - o[1]), self._peer(o[1] - o[2])
        p12 = self._peer(o[2] - o[1])
        msg, msg_rm, out0, out1 = R.trunc_party_r0(x.s0.v, x.s1.v, m, roles, slots, nonces)
        # round A, by message type: mk0 P0->P1, mk1 P1->P0, rt1 P2->P1, rm1 P2->P1
        rmk, rrt, rrm = torch.empty_like(msg), torch.empty_like(msg), torch.empty_like(msg_rm)
        self.comm.exchange([(msg[0], p01), (msg[1], p10), (msg[2], p21), (msg_rm[2], p21)],
                           [(rmk[1], p10), (rmk[0], p01), (rrt[1], p12), (rrm[1], p12)])
        w = R.trunc_party_r1(msg, rmk, rrt, rrm, out0, out1, bits, m, roles, slots, nonces)
        # round B: w0 P0->P1, w1 P1->P0; then z1 = w0 + w1 at both
        rw = torch.empty_like(w)
        self.comm.exchange([(w[0], p01), (w[1], p10)], [(rw[1], p10), (rw[0], p01)])
        out1[0].copy_(R.binary("add", R.RT(w[0], bits), R.RT(rw[0], bits)).data)
        out0[1].copy_(R.binary("add", R.RT(w[1], bits), R.RT(rw[1], bits)).data)
        nb = _nbytes(x.s0.v) // 3
        self.stats.record_round(3 * nb)
        self.stats.record_round(2 * nb)
        return PV(plc, R.RT(out0, bits)), PV(plc, R.RT(out1, bits))

    def party_share(self, plc, x, j, kind, n1, na):
        """Input sharing by member j: one kernel for every component's slots, then the
        owner's masked slot goes to its recipient -- x_{j+1} to P_{j+1} (its s0), or,
        mirrored (share_dir 2), x_j to P_{j+2} (its s1)."""
        bits = x.v.bits
        d = self.share_dir(plc, j)
        rel = [(c - j) % 3 for c in range(3)]
        slots = []
        for c in range(3):  # the PRF key: k_j (owner: own, P_{j+2}: next), mirrored k_{j+1}
            w = ({0: (0, 2), 1: (0, 2), 2: (1, 2)} if d == 1 else
                 {0: (1, 2), 1: (0, 2), 2: (0, 2)})[rel[c]]
            slots += [self._slot(plc, c, w[0]), self._slot(plc, c, w[1])]
        o = [self.offset(r) for r in plc.owners]
        jr = (j + d) % 3
        local = (o[jr] - o[j]) % self.N == 0  # the recipient of the owner's session is here
        if local:  # the kernel writes the owner's masked slot into the recipient's share too
            rel[j] += 4 * (1 + jr)
        out0, out1 = R.share_party(kind, x.v, 3, rel, slots, n1, na, mirror=d == 2)
        if not local:
            src, dst = (out1[j], out0[jr]) if d == 1 else (out0[j], out1[jr])
            self.comm.exchange([(src, self._peer(o[jr] - o[j]))],
                               [(dst, self._peer(o[j] - o[jr]))])
        self.stats.record_send(x.host, plc.owners[jr], _nbytes(x.v))
        return PV(plc, R.RT(out0, bits)), PV(plc, R.RT(out1, bits))

    def party_exchange(self, plc, specs):
        """Route per-party messages (parallel/party.py): party a's payload on this GPU goes
        to the GPU hosting party b of the same session; a message between two parties on
        the same GPU (offsets equal mod N) is the payload itself, no copy."""
        o = [self.offset(r) for r in plc.owners]
        got, sends, recvs = {}, [], []
        for name, a, b, t, like in specs:
            if (o[b] - o[a]) % self.N == 0:
                got[name] = t
                continue
            buf = like if isinstance(like, torch.Tensor) else torch.empty(
                like[0], dtype=like[1], device=self.device)
            sends.append((t, self._peer(o[b] - o[a])))
            recvs.append((buf, self._peer(o[a] - o[b])))
            got[name] = buf
        if sends:
            self.comm.exchange(sends, recvs)
        return got

    def party_dot_trunc_pre(self, plc, x, y, m, nonces):
        """The dealer's part of rep.dot_trunc's tail, issued before the GEMM of x . y
        (party.dealer_early); None for shapes other than a plain 2-D product."""
        from moose_amd.parallel import party

        xs, ys = x.s0.v.shape, y.s0.v.shape
        if len(xs) != 3 or len(ys) != 3:
            return None
        bits = x.bits
        shp = (3, xs[1], ys[2]) + ((2,) if bits == 128 else ())
        s0 = torch.empty(shp, dtype=torch.int64, device=self.device)
        s1 = torch.empty_like(s0)

        def run():
            return party.dealer_early(self, plc, [0, 1, 2], (shp[1:], torch.int64), bits, m,
                                      nonces, [s0[c] for c in range(3)],
                                      [s1[c] for c in range(3)], self._pair_ptrs(plc))

        # opt-in (DEALER_SIDE), one GPU: the dealer's keystream kernel needs nothing but
        # keys, so it can run on a side stream beside the GEMM; across GPUs it stays on the
        # step's stream (one RCCL communicator, one issue order)
        side = (DEALER_SIDE and self.device.type == "cuda"
                and getattr(self.comm, "world", 1) == 1)
        if side:
            main = torch.cuda.current_stream(self.device)
            st = self.side_stream()
            st.wait_stream(main)
            with torch.cuda.stream(st):
                pre = run()
            pre.event = torch.cuda.Event()
            pre.event.record(st)
            for t in [s0, s1] + [t for t in pre.rrt + pre.rrm if t is not None]:
                t.record_stream(main)
        else:
            pre = run()
        pre.stack = (s0, s1)
        return pre

    # rep.dot_trunc returns its product with the last reshare round pending (DeferredRep)
    defer_reshare = True

    def p_reveal_deferred(self, x, tail, host):
        """Reveal to the dealer P2 of a product whose round B is pending: w0, w1 go to P2
        (one round) and P2 sums z2 + z0 + w0 + w1 (fused into the decode).  None for other
        hosts (the generic reveal completes the shares first)."""
        plc = x.plc
        if host not in plc.owners or plc.owners.index(host) != 2:
            return None
        parts = tail.reveal_to_dealer()[2]
        return HV(host, R.opened(*[R.RT(t, x.bits) for t in parts]))

    def party_dot_trunc(self, plc, v, m, nonces, out=None, pre=None, defer=False):
        """rep.dot_trunc's zero share + reshare + TruncPr of the local products ``v`` with
        the reshare folded into TruncPr's first round (parallel/party.py); ``out``: optional
        (s0, s1) [3, ...] views (dense per component) written in place; ``pre``: the
        dealer's part from party_dot_trunc_pre (its buffers are the output)."""
        from moose_amd.parallel import party

        bits = v.v.bits
        data = v.v.data.contiguous()
        if pre is not None and pre.event is not None:  # the dealer part ran on a side stream
            torch.cuda.current_stream(self.device).wait_event(pre.event)
        if pre is not None:
            s0, s1 = pre.stack
        else:
            s0, s1 = out if out is not None else (torch.empty_like(data),
                                                  torch.empty_like(data))
        rb = party.dot_trunc_tail(self, plc, [0, 1, 2], [data[c] for c in range(3)], bits, m,
                                  nonces, [s0[c] for c in range(3)], [s1[c] for c in range(3)],
                                  self._pair_ptrs(plc), pre=pre, defer=defer)
        if defer:
            return PV(plc, R.RT(s0, bits)), PV(plc, R.RT(s1, bits)), rb
        return PV(plc, R.RT(s0, bits)), PV(plc, R.RT(s1, bits))

    # the single-GPU fused variants read other parties' data in-kernel: never used here
    p_mul_reshare = None
    p_zero_share_reshare = None

    def p_reveal(self, x, host):
        """Reveal to a member P_j: P_{j+1}'s second share (x_{j+2}) is the one message
        (party_exchange: a device buffer on another GPU, the share itself on this one),
        then one add3 kernel.  None for outsiders (generic path)."""
        plc = x.plc
        if host not in plc.owners:
            return None
        v0, v1 = x.s0.v, x.s1.v
        if not (isinstance(v0, R.RT) and isinstance(v1, R.RT)) or v0.bits not in (64, 128):
            return None
        j = plc.owners.index(host)
        j1 = (j + 1) % 3
        d1 = v1.data
        src = d1[j1] if d1[j1].is_contiguous() else d1[j1].contiguous()
        got = self.party_exchange(plc, [("reveal", j1, j, src, (tuple(src.shape), src.dtype))])
        self.stats.record_send(plc.owners[j1], host, _nbytes(v1) // 3)
        return HV(host, R.opened(R.RT(v0.data[j], v0.bits), R.RT(d1[j], v1.bits),
                                 R.RT(got["reveal"], v1.bits)))
    p_ks_level = None
    p_dot_zs_reshare = None
