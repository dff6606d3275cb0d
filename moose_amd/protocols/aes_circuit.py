"""Generator of an AES-128 encryption circuit in Bristol fashion.

The reference ships a pre-built 36,663-gate circuit (``bristol_fashion/aes_128.txt``);
this module *constructs* one from the cipher's algebra so no circuit file is needed:

* SubBytes = affine(x^254) in GF(2^8) (x^254 = x^-1, 0 -> 0) with the addition chain
  x^2, x^3 = x^2 x, x^12 = (x^3)^4, x^15 = x^12 x^3, x^240 = (x^15)^16,
  x^252 = x^240 x^12, x^254 = x^252 x^2 -- four GF(2^8) products (64 ANDs each),
  AND depth 4; squarings, MixColumns, ShiftRows, the key schedule and the S-box
  affine map are XOR/INV networks;
* the key schedule runs alongside the rounds, so the circuit's AND depth is 40.

Wire conventions (matching the reference's use of the circuit,
``encrypted/ops.rs:312-393``): inputs are the 128 key bits then the 128 block bits,
outputs the 128 ciphertext bits, all MSB-first in byte order (bit ``8*j`` is the most
significant bit of byte ``j`` of the big-endian 16-byte string).
"""
from __future__ import annotations

from functools import lru_cache
from typing import List

from moose_amd.protocols.bristol import Circuit
from moose_amd.protocols.bristol import Gate

_POLY = 0x11B


def _gf_mul_const(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= _POLY
        b >>= 1
    return r


class _Builder:
    def __init__(self, n_inputs: int):
        self.n = n_inputs
        self.gates: List[Gate] = []
        self._inv_cache = {}

    def _new(self, op, ins):
        w = self.n
        self.n += 1
        self.gates.append(Gate(op, tuple(ins), w))
        return w

    def xor(self, a, b):
        return self._new("XOR", (a, b))

    def and_(self, a, b):
        return self._new("AND", (a, b))

    def inv(self, a):
        return self._new("INV", (a,))

    def xor_many(self, ws):
        ws = list(ws)
        if not ws:
            raise ValueError("empty xor")
        acc = ws[0]
        for w in ws[1:]:
            acc = self.xor(acc, w)
        return acc

    def copy(self, a):
        return self._new("EQW", (a,))

    # -- GF(2^8) on bytes given as 8 wires, index 0 = least significant bit -----------
    def linear_byte(self, byte, matrix_cols, const=0):
        """out bit i = XOR_j [bit i of matrix_cols[j]] * byte[j]  ^ const bit i."""
        out = []
        for i in range(8):
            terms = [byte[j] for j in range(8) if (matrix_cols[j] >> i) & 1]
            w = self.xor_many(terms) if terms else None
            if (const >> i) & 1:
                w = self.inv(w) if w is not None else None
            if w is None:
                raise ValueError("constant-only output bit")
            out.append(w)
        return out

    def gf_mul(self, a, b):
        prod = [None] * 15
        for i in range(8):
            for j in range(8):
                t = self.and_(a[i], b[j])
                prod[i + j] = t if prod[i + j] is None else self.xor(prod[i + j], t)
        for k in range(14, 7, -1):  # reduce by x^8 = x^4 + x^3 + x + 1
            for s in (4, 3, 1, 0):
                prod[k - 8 + s] = self.xor(prod[k - 8 + s], prod[k])
        return prod[:8]

    def gf_pow2k(self, a, k):
        """a^(2^k): linear (Frobenius)."""
        cols = []
        for j in range(8):
            v = 1 << j
            for _ in range(k):
                v = _gf_mul_const(v, v)
            cols.append(v)
        return self.linear_byte(a, cols)

    def sbox(self, x):
        x2 = self.gf_pow2k(x, 1)
        x3 = self.gf_mul(x2, x)
        x12 = self.gf_pow2k(x3, 2)
        x15 = self.gf_mul(x12, x3)
        x240 = self.gf_pow2k(x15, 4)
        x252 = self.gf_mul(x240, x12)
        x254 = self.gf_mul(x252, x2)
        # affine: b_i ^ b_{i+4} ^ b_{i+5} ^ b_{i+6} ^ b_{i+7} ^ 0x63_i
        cols = []
        for j in range(8):
            c = 0
            for i in range(8):
                if j in (i, (i + 4) % 8, (i + 5) % 8, (i + 6) % 8, (i + 7) % 8):
                    c |= 1 << i
            cols.append(c)
        return self.linear_byte(x254, cols, 0x63)

    def xtime(self, a):
        return self.linear_byte(a, [_gf_mul_const(1 << j, 2) for j in range(8)])


def _msb_first_to_bytes(bits: List[int]) -> List[List[int]]:
    """128 wires MSB-first -> 16 bytes of 8 wires LSB-first."""
    return [[bits[8 * j + 7 - i] for i in range(8)] for j in range(16)]


def _bytes_to_msb_first(byts: List[List[int]]) -> List[int]:
    out = []
    for b in byts:
        out.extend(b[7 - i] for i in range(8))
    return out


@lru_cache(maxsize=1)
def aes128_circuit() -> Circuit:
    bld = _Builder(256)
    key = _msb_first_to_bytes(list(range(128)))
    state = _msb_first_to_bytes(list(range(128, 256)))
    # key schedule: words w[0..43] of 4 bytes
    w = [key[4 * i:4 * i + 4] for i in range(4)]
    rcon = 1
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = t[1:] + t[:1]
            t = [bld.sbox(b) for b in t]
            t[0] = [bld.inv(t[0][k]) if (rcon >> k) & 1 else t[0][k] for k in range(8)]
            rcon = _gf_mul_const(rcon, 2)
        w.append([[bld.xor(w[i - 4][b][k], t[b][k]) for k in range(8)] for b in range(4)])
    rk = [[byte for word in w[4 * r:4 * r + 4] for byte in word] for r in range(11)]

    def add_rk(s, r):
        return [[bld.xor(s[j][k], rk[r][j][k]) for k in range(8)] for j in range(16)]

    s = add_rk(state, 0)
    for r in range(1, 11):
        s = [bld.sbox(b) for b in s]
        s = [s[(j % 4) + 4 * (((j // 4) + (j % 4)) % 4)] for j in range(16)]  # ShiftRows
        if r < 10:
            ns = []
            for c in range(4):
                col = s[4 * c:4 * c + 4]
                x2 = [bld.xtime(b) for b in col]
                for row in range(4):
                    a0, a1, a2, a3 = (row + 0) % 4, (row + 1) % 4, (row + 2) % 4, (row + 3) % 4
                    # 2*a0 ^ 3*a1 ^ a2 ^ a3
                    ns.append([bld.xor_many([x2[a0][k], x2[a1][k], col[a1][k], col[a2][k],
                                             col[a3][k]]) for k in range(8)])
            s = ns
        s = add_rk(s, r)
    out_bits = _bytes_to_msb_first(s)
    # outputs must be the last 128 wires (Bristol convention)
    outs = [bld.copy(b) for b in out_bits]
    assert outs == list(range(bld.n - 128, bld.n))
    return Circuit(bld.n, [128, 128], [128], bld.gates)
