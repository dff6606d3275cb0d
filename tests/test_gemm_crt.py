"""Multi-modular (CRT) ring GEMM (csrc/gemm_crt.hip).

CPU: the moduli choice and the host tables are checked by re-running the kernels'
arithmetic (byte-weighted residues, centered reductions, CRT reconstruction with the
rounded quotient) in numpy on random and worst-case operands against exact python-int
products.  GPU: the kernels, forced on, are bit-exact against the host ring GEMM and the
limb GEMM, including worst-case operands at the largest inner dimension of one call."""
import math

import numpy as np
import pytest
import torch

from moose_amd.ops import native as nat
from moose_amd.ops import ring as R


def _tables(words, n):
    lib = nat.lib()
    p = np.zeros(n, np.int32)
    wa = np.zeros((n, 16), np.uint8)
    wb = np.zeros((n, 16), np.uint8)
    nega = np.zeros(n, np.int32)
    negb = np.zeros(n, np.int32)
    W = np.zeros((n, 8), np.uint16)
    Mw = np.zeros(8, np.uint16)
    ptr = lambda a: a.ctypes.data_as(nat.ctypes.c_void_p)  # noqa: E731
    assert lib.mx_crt_tables(words, n, ptr(p), ptr(wa), ptr(wb), ptr(nega), ptr(negb), ptr(W),
                             ptr(Mw)) == 0
    join = lambda ws: sum(int(v) << (16 * k) for k, v in enumerate(ws))  # noqa: E731
    return dict(p=p.astype(np.int64), wa=wa.astype(np.int64), wb=wb.astype(np.int64),
                nega=nega.astype(np.int64), negb=negb.astype(np.int64),
                W=[join(w) for w in W], Mw=join(Mw))


def _centered(s, p):
    return (s + p // 2) % p - p // 2


def _residues(vals, bits, t, side):
    """int8 residues [len(vals), n] exactly as k_crt_prep computes them."""
    nb = bits // 8
    v = np.array([[(x >> (8 * j)) & 0xFF for j in range(nb)] for x in vals], dtype=np.int64)
    negbit = np.array([x >> (bits - 1) for x in vals], dtype=np.int64)
    w = t["wa" if side == "a" else "wb"][:, :nb]
    neg = t["nega" if side == "a" else "negb"]
    s = v @ w.T + negbit[:, None] * neg[None, :]
    out = _centered(s, t["p"][None, :])
    out[:, 0] = ((v[:, 0] * neg[0]) & 0xFF) - (((v[:, 0] * neg[0]) & 0x80) << 1)  # p = 256
    return out


def _crt_dot(A, B, bits):
    """A [M][K], B [K][N] python ints mod 2^bits -> the kernels' result."""
    words = bits // 64
    K = len(B)
    n = nat.lib().mx_crt_moduli(words, K)
    t = _tables(words, n)
    M, N = len(A), len(B[0])
    ra = _residues([x for row in A for x in row], bits, t, "a").reshape(M, K, n)
    rb = _residues([x for row in B for x in row], bits, t, "b").reshape(K, N, n)
    acc = np.einsum("mki,kni->mni", ra, rb)
    c = _centered(acc, t["p"][None, None, :])
    out = []
    for m in range(M):
        row = []
        for j in range(N):
            ci = [int(v) for v in c[m, j]]
            q = round(sum(ci[i] / int(t["p"][i]) for i in range(n)))
            z = sum(ci[i] * t["W"][i] for i in range(n)) - q * t["Mw"]
            row.append(z % (1 << bits))
        out.append(row)
    return out


def _exact(A, B, bits):
    K = len(B)
    return [[sum(A[m][k] * B[k][j] for k in range(K)) % (1 << bits) for j in range(len(B[0]))]
            for m in range(len(A))]


def test_moduli_counts_and_bound():
    lib = nat.lib()
    assert lib.mx_crt_moduli(2, 8192) == 36  # vs 136 limb-pair GEMMs (37 with 256, 255, ...)
    assert lib.mx_crt_moduli(1, 8192) == 18  # vs 36
    for words in (1, 2):
        for kp in (1, 100, 8192, 32768):
            n = lib.mx_crt_moduli(words, kp)
            t = _tables(words, n)
            ps = [int(p) for p in t["p"]]
            assert all(math.gcd(a, b) == 1 for i, a in enumerate(ps) for b in ps[i + 1:])
            M = math.prod(ps)
            zmax = kp * (1 << (2 * 64 * words - 2))
            assert zmax <= 0.45 * M
            # one modulus fewer would not do
            assert kp == 1 or zmax > 0.45 * math.prod(ps[:-1]) or n == 1


@pytest.mark.parametrize("bits", [64, 128])
def test_crt_arithmetic_random(bits):
    rng = np.random.default_rng(bits)
    M, K, N = 3, 37, 4
    A = [[int.from_bytes(rng.bytes(bits // 8), "little") for _ in range(K)] for _ in range(M)]
    B = [[int.from_bytes(rng.bytes(bits // 8), "little") for _ in range(N)] for _ in range(K)]
    assert _crt_dot(A, B, bits) == _exact(A, B, bits)


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("a,b", [("min", "min"), ("min", "max"), ("max", "max")])
def test_crt_arithmetic_worst_case(bits, a, b):
    """|Z| at its bound: every product at +-2^(2w-2), K' = 8192 (one bench-size call)."""
    K = 8192
    val = {"min": 1 << (bits - 1), "max": (1 << (bits - 1)) - 1}
    A = [[val[a]] * K]
    B = [[val[b]] for _ in range(K)]
    assert _crt_dot(A, B, bits) == _exact(A, B, bits)


@pytest.mark.parametrize("bits", [64, 128])
def test_dot4_reconstruction_tables(bits):
    """k_crt_recon16d's digit tables: W_i mod 2^w and round(2^24 / p_i) recompose from their
    signed base-256 digits, and the integer quotient estimate round(sum c_i R_i / 2^24)
    reconstructs random products Z at the |Z| <= 0.45 M bound exactly."""
    lib = nat.lib()
    words = bits // 64
    n = lib.mx_crt_moduli(words, 8192)
    t = _tables(words, n)
    wd = np.zeros(12 * 16, np.uint32)
    rd = np.zeros(12 * 3, np.uint32)
    ptr = lambda a: a.ctypes.data_as(nat.ctypes.c_void_p)  # noqa: E731
    assert lib.mx_crt_tables4(words, n, ptr(wd), ptr(rd)) == (n + 3) // 4

    def digit(word, u):
        b = (int(word) >> (8 * u)) & 0xFF
        return b - 256 if b >= 128 else b

    ps = [int(p) for p in t["p"]]
    R = []
    for i in range(n):
        W = sum(digit(wd[(i // 4) * 16 + d], i % 4) * 256**d for d in range(bits // 8))
        assert W % (1 << bits) == t["W"][i] % (1 << bits)
        R.append(sum(digit(rd[(i // 4) * 3 + d], i % 4) * 256**d for d in range(3)))
        assert R[-1] == round((1 << 24) / ps[i])
    M = math.prod(ps)
    inv = [pow(M // p, -1, p) for p in ps]
    rng = np.random.default_rng(bits)
    for trial in range(200):
        frac = (rng.random() * 2 - 1) * 0.45 if trial > 1 else (0.45, -0.45)[trial]
        Z = int(frac * M)
        c = [_centered(Z * inv[i], ps[i]) for i in range(n)]
        q = ((sum(ci * ri for ci, ri in zip(c, R))) + (1 << 23)) >> 24
        z = (sum(ci * wi for ci, wi in zip(c, t["W"])) - q * t["Mw"]) % (1 << bits)
        assert z == Z % (1 << bits)


# --- GPU ------------------------------------------------------------------------------------
def rand_rt(shape, bits, seed):
    g = torch.Generator().manual_seed(seed)
    lo = torch.randint(-(2**63), 2**63 - 1, shape + ((2,) if bits == 128 else ()),
                       generator=g, dtype=torch.int64)
    return R.RT(lo, bits)


def gpu(x):
    return R.RT(x.data.cuda(), x.bits)


def same(a, b):
    assert a.bits == b.bits
    assert torch.equal(a.data.cpu(), b.data.cpu())


class _crt:
    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        nat.lib().mx_set_gemm_crt(self.mode)

    def __exit__(self, *a):
        nat.lib().mx_set_gemm_crt(0)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("shape", [(3, 5, 4), (70, 130, 96), (300, 520, 270)])
def test_gpu_crt_gemm_matches_host(bits, shape):
    M, K, N = shape
    a, b = rand_rt((2, M, K), bits, 10), rand_rt((2, K, N), bits, 11)
    with _crt(1):
        d = R.dot(gpu(a), gpu(b), nb=1)
    same(R.dot(a, b, nb=1), d)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
def test_gpu_crt_cross_matches_host(bits):
    M, K, N = 273, 260, 300
    xs = [rand_rt((3, M, K), bits, 20 + i) for i in range(2)]
    ys = [rand_rt((3, K, N), bits, 30 + i) for i in range(2)]
    h = R.dot_cross(xs[0], xs[1], ys[0], ys[1], nb=1)
    with _crt(1):
        d = R.dot_cross(gpu(xs[0]), gpu(xs[1]), gpu(ys[0]), gpu(ys[1]), nb=1)
    same(h, d)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
def test_gpu_crt_matches_limb_gemm_large(bits):
    M, K, N = 512, 2048, 768
    xs = [gpu(rand_rt((3, M, K), bits, 50 + i)) for i in range(2)]
    ys = [gpu(rand_rt((3, K, N), bits, 60 + i)) for i in range(2)]
    with _crt(1):
        c = R.dot_cross(*xs, *ys, nb=1)
    with _crt(2):
        lmb = R.dot_cross(*xs, *ys, nb=1)
    same(c, lmb)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
def test_gpu_crt_long_k_accumulates(bits):
    # K above one call's exact limit: the caller splits K and accumulates into C
    a, b = rand_rt((1, 64, 9000), bits, 40), rand_rt((1, 9000, 80), bits, 41)
    with _crt(1):
        d = R.dot(gpu(a), gpu(b), nb=1)
    same(R.dot(a, b, nb=1), d)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("va,vb", [("min", "min"), ("min", "max"), ("max", "max")])
def test_gpu_crt_worst_case_at_max_k(bits, va, vb):
    """Mode 1 at K' = 8192 (the bench's call) with every operand at an extreme signed value."""
    K = 4096
    val = {"min": 1 << (bits - 1), "max": (1 << (bits - 1)) - 1}
    mask = (1 << bits) - 1

    def full(shape, v):
        return R.fill(shape, v, bits, torch.device("cuda"))

    x0, x1 = full((3, 64, K), val[va]), full((3, 64, K), val[va])
    y0, y1 = full((3, K, 40), val[vb]), full((3, K, 40), val[vb])
    with _crt(1):
        c = R.dot_cross(x0, x1, y0, y1, nb=1)
    # x0.(y0 + y1) + x1.y0 with every entry equal: K a (2b mod 2^w) + K a b
    a, b = val[va], val[vb]
    want = (K * a * ((2 * b) & mask) + K * a * b) & mask
    got = R.to_ints(c)
    assert (got == want).all()


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
def test_gpu_crt_prepared_b_rows(bits):
    M, K, N = 600, 300, 280
    xs = [rand_rt((3, M, K), bits, 70 + i) for i in range(2)]
    ys = [rand_rt((3, K, N), bits, 80 + i) for i in range(2)]
    want = R.dot_cross(xs[0], xs[1], ys[0], ys[1], nb=1)
    with _crt(1):
        pb = R.PreparedCross(gpu(ys[0]), gpu(ys[1]))
        parts = [R.dot_cross_rows(gpu(xs[0]), gpu(xs[1]), r0, min(M, r0 + 256), pb)
                 for r0 in range(0, M, 256)]
    got = torch.cat([p.data.cpu() for p in parts], dim=1)
    assert torch.equal(got, want.data)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("crt", [1, 2])
@pytest.mark.parametrize("both", [False, True])
def test_gpu_dot_cross_broadcast_views(bits, crt, both):
    """[3, k, M, K] stride-0 stacks of one operand (fixedpoint.dot_many on k uses of the same
    values) go to the strided GEMM without a copy -- the CRT path prepares a broadcast
    operand's residues once; equal to the materialised product."""
    k, M, K, N = 5, 300, 270, 260
    xs = [gpu(rand_rt((3, M, K), bits, 90 + i)) for i in range(2)]

    def view(t):
        d = t.data.unsqueeze(1)
        return R.RT(d.expand((3, k) + tuple(d.shape[2:])), bits)

    if both:
        ys = [view(gpu(rand_rt((3, K, N), bits, 95 + i))) for i in range(2)]
    else:
        ys = [gpu(rand_rt((3, 1, K, N), bits, 95 + i)) for i in range(2)]
        ys = [R.RT(torch.cat([y.data] * k, dim=1), bits) for y in ys]  # a real stack for y
    dense = [R.RT(y.data.contiguous(), bits) for y in ys]
    with _crt(crt):
        got = R.dot_cross(view(xs[0]), view(xs[1]), ys[0], ys[1], nb=2)
        want = R.dot_cross(R.RT(view(xs[0]).data.contiguous(), bits),
                           R.RT(view(xs[1]).data.contiguous(), bits), *dense, nb=2)
    same(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("K", [320, 300])
def test_gpu_dot_cross_pair_rolled(bits, K):
    """An RSS pair (x1 = x0 rolled by one party) through the rolled CRT GEMM (each share's
    residues prepared once) equals the two-operand product; K not a multiple of the k-block
    falls back (None).  Also with a prepared B' and row blocks."""
    M, N = 300, 280
    x0 = gpu(rand_rt((3, M, K), bits, 110))
    x1 = R.RT(torch.roll(x0.data, -1, dims=0).contiguous(), bits)
    ys = [gpu(rand_rt((3, K, N), bits, 111 + i)) for i in range(2)]
    with _crt(1):
        want = R.dot_cross(x0, x1, *ys, nb=1)
        got = R.dot_cross_pair(x0, ys[0], ys[1], 1)
        pb = R.PreparedCross(*ys)
        rows = [R.dot_cross_pair(x0, None, None, 1, pb=pb, r0=r0, r1=min(M, r0 + 128))
                for r0 in range(0, M, 128)]
    if K % 64:
        assert got is None and all(r is None for r in rows)
        return
    same(want, got)
    assert torch.equal(torch.cat([r.data for r in rows], dim=1).cpu(), want.data.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["6", "8", "12", "14", "16"])
def test_gpu_crt_bench_tiling_matches_limb_gemm(variant, monkeypatch):
    """The bench's tile grid: many 256x256 tiles in both directions (GROUPM remap over 8 x 8
    tiles per party and modulus), K' = 8192 (mode 1), Z_2^128 -- bit-exact against the limb
    GEMM, for the plain cross GEMM and the rolled-pair form the stacked session runs."""
    monkeypatch.setenv("MOOSEX_CRT_KERNEL", variant)
    bits, M, K, N = 128, 2048, 4096, 2048
    x0 = gpu(rand_rt((3, M, K), bits, 90))
    ys = [gpu(rand_rt((3, K, N), bits, 91 + i)) for i in range(2)]
    x1 = R.RT(torch.roll(x0.data, -1, dims=0), bits)  # s1[p] = s0[p + 1]
    with _crt(2):
        want = R.dot_cross(x0, x1, *ys, nb=1)
    with _crt(1):
        got = R.dot_cross(x0, x1, *ys, nb=1)
        rolled = R.dot_cross_pair(x0, ys[0], ys[1], 1)
    same(want, got)
    assert rolled is not None
    same(want, rolled)
