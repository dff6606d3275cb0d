"""Bristol-fashion boolean circuits, levelised for batched secure evaluation.

Parity: reference ``moose/src/bristol_fashion/mod.rs`` (``Circuit`` :95-131, the nom
parser :133, and ``aes128`` :16-93 which evaluates the circuit gate by gate on any
placement implementing Xor/And/Neg).

MI355X design: gate-by-gate evaluation would issue ~36k tiny kernels and one network
round per AND gate.  Instead :class:`LevelledCircuit` compiles the circuit once:

* every wire is rewritten as an affine GF(2) combination of *base* wires (circuit
  inputs and AND-gate outputs) plus a constant -- XOR/INV/EQW chains collapse;
* AND gates are grouped by AND-depth; a level is evaluated as ONE sparse GF(2)
  matrix product per party (``M_left @ base``, ``M_right @ base``, exact in fp32 then
  ``& 1``) followed by ONE batched secret AND (one communication round for the whole
  level, all blocks of the batch at once);
* the outputs are one more affine map.

So a circuit costs ``AND-depth`` rounds and ``2 * AND-depth + 1`` sparse GEMMs per
party regardless of its gate count.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List
from typing import Sequence
from typing import Tuple

import numpy as np
import torch

from moose_amd.ops import ring as R


@dataclass
class Gate:
    op: str  # XOR | AND | INV | EQW | EQ
    ins: Tuple[int, ...]
    out: int


@dataclass
class Circuit:
    num_wires: int
    input_sizes: List[int]
    output_sizes: List[int]
    gates: List[Gate]

    @property
    def num_inputs(self):
        return sum(self.input_sizes)

    @property
    def num_outputs(self):
        return sum(self.output_sizes)

    def stats(self):
        c = {}
        for g in self.gates:
            c[g.op] = c.get(g.op, 0) + 1
        return c

    def to_bristol(self) -> str:
        lines = [f"{len(self.gates)} {self.num_wires}",
                 " ".join([str(len(self.input_sizes))] + [str(s) for s in self.input_sizes]),
                 " ".join([str(len(self.output_sizes))] + [str(s) for s in self.output_sizes]),
                 ""]
        for g in self.gates:
            if g.op == "EQ":
                lines.append(f"1 1 {g.ins[0]} {g.out} EQ")
            else:
                lines.append(f"{len(g.ins)} 1 {' '.join(map(str, g.ins))} {g.out} {g.op}")
        return "\n".join(lines) + "\n"


def parse_bristol(text: str) -> Circuit:
    """Parse the Bristol-fashion format: header ``#gates #wires``, input and output
    size lines, then one gate per line ``nin nout in... out... OP``."""
    toks = [ln.split() for ln in text.strip().splitlines() if ln.strip()]
    ngates, nwires = int(toks[0][0]), int(toks[0][1])
    ins = [int(x) for x in toks[1][1:1 + int(toks[1][0])]]
    outs = [int(x) for x in toks[2][1:1 + int(toks[2][0])]]
    gates = []
    for t in toks[3:3 + ngates]:
        nin, nout = int(t[0]), int(t[1])
        op = t[-1]
        wires = [int(x) for x in t[2:2 + nin + nout]]
        if op not in ("XOR", "AND", "INV", "EQW", "EQ"):
            raise ValueError(f"unsupported gate {op}")
        gates.append(Gate(op, tuple(wires[:nin]), wires[nin]))
    if len(gates) != ngates:
        raise ValueError("truncated circuit")
    return Circuit(nwires, ins, outs, gates)


class LevelledCircuit:
    """See module doc.  Base wires: ``[inputs (n_in), AND outputs of level 1, ...]``."""

    def __init__(self, c: Circuit):
        self.circuit = c
        n_in = c.num_inputs
        # pass 1: AND depth of every wire; AND gates grouped by level (gate order)
        depth = [0] * c.num_wires
        and_by_level: List[List[Gate]] = []
        for g in c.gates:
            d = max(depth[i] for i in g.ins)
            if g.op == "AND":
                d += 1
                while len(and_by_level) < d:
                    and_by_level.append([])
                and_by_level[d - 1].append(g)
            depth[g.out] = d
        # level-major base indices of AND outputs
        base_of = {}
        nxt = n_in
        for lvl in and_by_level:
            for g in lvl:
                base_of[g.out] = nxt
                nxt += 1
        # pass 2: every wire as (set of base indices, constant bit)
        expr = [None] * c.num_wires
        for w in range(n_in):
            expr[w] = (frozenset([w]), 0)
        for g in c.gates:
            if g.op == "AND":
                expr[g.out] = (frozenset([base_of[g.out]]), 0)
            elif g.op == "XOR":
                a, b = expr[g.ins[0]], expr[g.ins[1]]
                expr[g.out] = (a[0] ^ b[0], a[1] ^ b[1])
            elif g.op == "INV":
                a = expr[g.ins[0]]
                expr[g.out] = (a[0], a[1] ^ 1)
            else:  # EQW / EQ: wire copy
                expr[g.out] = expr[g.ins[0]]
        self.n_in = n_in
        self.n_base = nxt
        self.depth = len(and_by_level)
        self.levels = []  # per level: (left affine, right affine, base offset, count)
        off = n_in
        for lvl in and_by_level:
            left = _SparseAffine([expr[g.ins[0]] for g in lvl], off)
            right = _SparseAffine([expr[g.ins[1]] for g in lvl], off)
            self.levels.append((left, right, off, len(lvl)))
            off += len(lvl)
        out_wires = list(range(c.num_wires - c.num_outputs, c.num_wires))
        self.outputs = _SparseAffine([expr[w] for w in out_wires], self.n_base)
        self.and_count = off - n_in

    # -- evaluation -------------------------------------------------------------------
    def eval_plain(self, inputs: torch.Tensor) -> torch.Tensor:
        """``inputs``: uint8 {0,1} of shape [n_in, *batch] -> [n_out, *batch]."""
        base = inputs.to(torch.uint8)
        for left, right, _, _ in self.levels:
            a = left.apply(base)
            b = right.apply(base)
            base = torch.cat([base, a & b], dim=0)
        return self.outputs.apply(base)

    def eval_shared(self, sess, x):
        """Secure evaluation on a boolean bit sharing ``x`` (RepTensor, bits=1) of shape
        [n_in, *batch]: one batched AND round per level."""
        from moose_amd.protocols import replicated as rep

        base = x
        for left, right, _, _ in self.levels:
            a = _affine_shared(sess, left, base)
            b = _affine_shared(sess, right, base)
            ab = rep.and_(sess, a, b)
            base = rep.RepTensor(base.plc, 1, "bool",
                                 sess.p("Concat", base.plc, base.s0, ab.s0, axis=0),
                                 sess.p("Concat", base.plc, base.s1, ab.s1, axis=0))
        return _affine_shared(sess, self.outputs, base)


class _SparseAffine:
    """rows[i] = (set of base indices, constant): out_i = XOR_{j in set} base_j ^ c_i."""

    def __init__(self, rows: Sequence[Tuple[frozenset, int]], ncols: int):
        self.nrows = len(rows)
        self.ncols = ncols
        ri, ci = [], []
        for i, (s, _) in enumerate(rows):
            for j in s:
                if j >= ncols:
                    raise ValueError("affine row refers to a later base wire")
                ri.append(i)
                ci.append(j)
        self.row_idx = np.asarray(ri, dtype=np.int64)
        self.col_idx = np.asarray(ci, dtype=np.int64)
        self.const = np.asarray([c for (_, c) in rows], dtype=np.uint8)
        self._cache = {}

    def matrix(self, device):
        m = self._cache.get(device)
        if m is None:
            idx = R.to_device(torch.as_tensor(np.stack([self.row_idx, self.col_idx])), device)
            vals = torch.ones(len(self.row_idx), dtype=torch.float32, device=device)
            m = torch.sparse_coo_tensor(idx, vals, (self.nrows, self.ncols)).coalesce()
            self._cache[device] = m
        return m

    def linear(self, base: torch.Tensor) -> torch.Tensor:
        """XOR part only (no constant): sparse fp32 GEMM over the flattened batch."""
        shp = base.shape
        b2 = base[: self.ncols].reshape(self.ncols, -1).to(torch.float32)
        y = torch.sparse.mm(self.matrix(base.device), b2)
        return (y.to(torch.int32) & 1).to(torch.uint8).reshape((self.nrows,) + tuple(shp[1:]))

    def apply(self, base: torch.Tensor) -> torch.Tensor:
        y = self.linear(base)
        c = R.to_device(torch.as_tensor(self.const), base.device).reshape((-1,) + (1,) * (y.dim() - 1))
        return y ^ c


def _affine_shared(sess, aff: _SparseAffine, x):
    """Share-wise GF(2) affine map: the linear part on every share, the constant on
    slot 0 only (a public XOR)."""
    from moose_amd.ops import ring as R
    from moose_amd.protocols import replicated as rep

    s0 = sess.p("BitAffine", x.plc, x.s0, aff=aff)
    s1 = sess.p("BitAffine", x.plc, x.s1, aff=aff)
    y = rep.RepTensor(x.plc, 1, "bool", s0, s1)
    if aff.const.any():
        shape = (aff.nrows,) + (1,) * (len(sess.p_shape(x.s0)) - 1)
        c = R.RT(R.to_device(torch.as_tensor(aff.const), sess.device).reshape(shape), 1)
        y = rep.add_public(sess, y, c)
    return y
