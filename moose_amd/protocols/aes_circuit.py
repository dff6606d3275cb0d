"""Generator of an AES-128 encryption circuit in Bristol fashion.

The reference ships a pre-built 36,663-gate circuit (``bristol_fashion/aes_128.txt``);
this module *constructs* one from the cipher's algebra so no circuit file is needed:

* SubBytes is Boyar and Peralta's 32-AND S-box circuit (_Builder.sbox), so the whole
  cipher has 200 x 32 = 6,400 AND gates (10 rounds x 16 S-boxes + 40 in the key
  schedule) -- the AND count of the reference's circuit, and the only gates that cost
  communication in MPC; MixColumns, ShiftRows, the key schedule and the S-box affine
  layers are XOR/INV networks;
* the key schedule runs alongside the rounds; AND depth 6 per S-box layer.

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
        """SubBytes with 32 AND gates: the Boyar-Peralta circuit (a linear top layer
        8 -> 22 wires, a 32-AND nonlinear core -- the GF(2^4)-tower inversion --, a linear
        bottom layer 18 -> 8 with the affine constant folded into four XNORs); AND depth 6.
        Checked against the S-box table on all 256 inputs in tests/test_aes.py."""
        X, A, N = self.xor, self.and_, self.inv
        x0, x1, x2, x3, x4, x5, x6, x7 = (x[7 - i] for i in range(8))  # x0 = msb
        y14 = X(x3, x5); y13 = X(x0, x6); y9 = X(x0, x3); y8 = X(x0, x5)  # noqa: E702
        t0 = X(x1, x2); y1 = X(t0, x7); y4 = X(y1, x3); y12 = X(y13, y14)  # noqa: E702
        y2 = X(y1, x0); y5 = X(y1, x6); y3 = X(y5, y8); t1 = X(x4, y12)  # noqa: E702
        y15 = X(t1, x5); y20 = X(t1, x1); y6 = X(y15, x7); y10 = X(y15, t0)  # noqa: E702
        y11 = X(y20, y9); y7 = X(x7, y11); y17 = X(y10, y11); y19 = X(y10, y8)  # noqa: E702
        y16 = X(t0, y11); y21 = X(y13, y16); y18 = X(x0, y16)  # noqa: E702
        t2 = A(y12, y15); t3 = A(y3, y6); t4 = X(t3, t2); t5 = A(y4, x7)  # noqa: E702
        t6 = X(t5, t2); t7 = A(y13, y16); t8 = A(y5, y1); t9 = X(t8, t7)  # noqa: E702
        t10 = A(y2, y7); t11 = X(t10, t7); t12 = A(y9, y11); t13 = A(y14, y17)  # noqa: E702
        t14 = X(t13, t12); t15 = A(y8, y10); t16 = X(t15, t12); t17 = X(t4, t14)  # noqa: E702
        t18 = X(t6, t16); t19 = X(t9, t14); t20 = X(t11, t16); t21 = X(t17, y20)  # noqa: E702
        t22 = X(t18, y19); t23 = X(t19, y21); t24 = X(t20, y18); t25 = X(t21, t22)  # noqa: E702
        t26 = A(t21, t23); t27 = X(t24, t26); t28 = A(t25, t27); t29 = X(t28, t22)  # noqa: E702
        t30 = X(t23, t24); t31 = X(t22, t26); t32 = A(t31, t30); t33 = X(t32, t24)  # noqa: E702
        t34 = X(t23, t33); t35 = X(t27, t33); t36 = A(t24, t35); t37 = X(t36, t34)  # noqa: E702
        t38 = X(t27, t36); t39 = A(t29, t38); t40 = X(t25, t39); t41 = X(t40, t37)  # noqa: E702
        t42 = X(t29, t33); t43 = X(t29, t40); t44 = X(t33, t37); t45 = X(t42, t41)  # noqa: E702
        z0 = A(t44, y15); z1 = A(t37, y6); z2 = A(t33, x7); z3 = A(t43, y16)  # noqa: E702
        z4 = A(t40, y1); z5 = A(t29, y7); z6 = A(t42, y11); z7 = A(t45, y17)  # noqa: E702
        z8 = A(t41, y10); z9 = A(t44, y12); z10 = A(t37, y3); z11 = A(t33, y4)  # noqa: E702
        z12 = A(t43, y13); z13 = A(t40, y5); z14 = A(t29, y2); z15 = A(t42, y9)  # noqa: E702
        z16 = A(t45, y14); z17 = A(t41, y8)  # noqa: E702
        t46 = X(z15, z16); t47 = X(z10, z11); t48 = X(z5, z13); t49 = X(z9, z10)  # noqa: E702
        t50 = X(z2, z12); t51 = X(z2, z5); t52 = X(z7, z8); t53 = X(z0, z3)  # noqa: E702
        t54 = X(z6, z7); t55 = X(z16, z17); t56 = X(z12, t48); t57 = X(t50, t53)  # noqa: E702
        t58 = X(z4, t46); t59 = X(z3, t54); t60 = X(t46, t57); t61 = X(z14, t57)  # noqa: E702
        t62 = X(t52, t58); t63 = X(t49, t58); t64 = X(z4, t59); t65 = X(t61, t62)  # noqa: E702
        t66 = X(z1, t63); s0 = X(t59, t63); s6 = N(X(t56, t62)); s7 = N(X(t48, t60))  # noqa: E702
        t67 = X(t64, t65); s3 = X(t53, t66); s4 = X(t51, t66); s5 = X(t47, t65)  # noqa: E702
        s1 = N(X(t64, s3)); s2 = N(X(t55, t67))  # noqa: E702
        return [s7, s6, s5, s4, s3, s2, s1, s0]  # lsb first

    def sbox_algebraic(self, x):
        """The round-1 S-box: affine(x^254) by four schoolbook GF(2^8) products (256 ANDs,
        AND depth 4).  Kept for before/after measurements (MOOSEX_AES_SBOX=algebraic)."""
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
    import os

    bld = _Builder(256)
    if os.environ.get("MOOSEX_AES_SBOX") == "algebraic":
        bld.sbox = bld.sbox_algebraic
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
