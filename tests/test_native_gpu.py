"""Bit-exact checks of every gfx950 ring kernel against the host (CPU) kernels, which
are in turn checked against python-int arithmetic in test_ring_cpu.py."""
import random

import pytest
import torch

from moose_amd.ops import native as nat
from moose_amd.ops import ring as R

pytestmark = pytest.mark.gpu

M64, M128 = (1 << 64) - 1, (1 << 128) - 1


def rand_rt(shape, bits, seed):
    g = torch.Generator().manual_seed(seed)
    if bits == 1:
        return R.RT(torch.randint(0, 2, shape, generator=g, dtype=torch.uint8), 1)
    lo = torch.randint(-(2**63), 2**63 - 1, shape + ((2,) if bits == 128 else ()),
                       generator=g, dtype=torch.int64)
    return R.RT(lo, bits)


def gpu(x):
    return R.RT(x.data.cuda(), x.bits)


def same(a, b):
    assert a.bits == b.bits
    assert torch.equal(a.data.cpu(), b.data.cpu())


def test_library_is_native_and_gpu_visible():
    assert nat.lib().mx_device_count() >= 1
    assert nat.loaded_path().endswith("libmoosex.so")


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("op", ["add", "sub", "mul", "and", "or", "xor"])
def test_binary(bits, op):
    a, b = rand_rt((1000,), bits, 1), rand_rt((1000,), bits, 2)
    same(R.binary(op, a, b), R.binary(op, gpu(a), gpu(b)))


@pytest.mark.parametrize("bits", [64, 128])
def test_unary_and_compare(bits):
    a, b = rand_rt((777,), bits, 3), rand_rt((777,), bits, 4)
    for op in ("neg", "not"):
        same(R.unary(op, a), R.unary(op, gpu(a)))
    for k in (0, 1, 31, 63, bits - 1):
        same(a.shl(k), gpu(a).shl(k))
        same(a.shr(k), gpu(a).shr(k))
    for op in ("lt", "gt", "eq"):
        same(R.compare(op, a, b), R.compare(op, gpu(a), gpu(b)))


@pytest.mark.parametrize("bits", [64, 128])
def test_encode_decode_sum(bits):
    x = torch.randn(513, dtype=torch.float64) * 1000
    same(R.encode(x, 23, bits), R.encode(x.cuda(), 23, bits))
    e = R.encode(x, 23, bits)
    assert torch.equal(R.decode(e, 23), R.decode(gpu(e), 23).cpu())
    a = rand_rt((7, 300, 5), bits, 5)
    for ax in (0, 1, 2):
        same(R.sum(a, ax), R.sum(gpu(a), ax))
    big = rand_rt((4096, 3), bits, 6)
    same(R.sum(big, 0), R.sum(gpu(big), 0))


def test_prg_matches_host():
    key = bytes(range(16))
    for n in (1, 15, 16, 17, 1000, 4099):
        h = R.prg_bytes(key, 123, n, "cpu")
        d = R.prg_bytes(key, 123, n, "cuda")
        assert torch.equal(h, d.cpu())


@pytest.mark.parametrize("bits", [1, 64, 128])
@pytest.mark.parametrize("kind", ["arith", "bool"])
def test_rss_cross_fused(bits, kind):
    if bits == 1 and kind == "arith":
        pytest.skip("bits use the boolean flavour")
    keys = [bytes([i] * 16) for i in range(3)]
    keys = keys + keys[:1]
    xs = [rand_rt((3, 1001), bits, s) for s in range(4)]
    h = R.rss_cross(kind, *xs, keys, 99, 3)
    d = R.rss_cross(kind, *[gpu(x) for x in xs], keys, 99, 3)
    same(h, d)
    z1 = R.prf_expand(keys[:3], 5, (333,), bits, "cpu")
    z2 = R.prf_expand(keys[:3], 5, (333,), bits, "cuda")
    same(z1, z2)


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("shape", [(3, 5, 4), (64, 64, 64), (70, 130, 96), (128, 256, 192)])
def test_gemm_matches_host(bits, shape):
    M, K, N = shape
    a, b = rand_rt((2, M, K), bits, 10), rand_rt((2, K, N), bits, 11)
    same(R.dot(a, b, nb=1), R.dot(gpu(a), gpu(b), nb=1))


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("shape", [(100, 128, 1), (128, 100, 1), (7, 300, 3), (129, 65, 4),
                                   (1, 1, 1), (5, 1000, 2)])
def test_skinny_gemm_matches_host(bits, shape):
    """N <= 4: the wave-per-row product (k_gemv_valu), batched and single, plain and the
    RSS cross form, equal to the host's."""
    M, K, N = shape
    a, b = rand_rt((2, M, K), bits, 12), rand_rt((2, K, N), bits, 13)
    same(R.dot(a, b, nb=1), R.dot(gpu(a), gpu(b), nb=1))
    a1, b1 = rand_rt((M, K), bits, 14), rand_rt((K, N), bits, 15)
    same(R.dot(a1, b1), R.dot(gpu(a1), gpu(b1)))
    xs = [rand_rt((3, M, K), bits, 40 + i) for i in range(2)]
    ys = [rand_rt((3, K, N), bits, 50 + i) for i in range(2)]
    same(R.dot_cross(xs[0], xs[1], ys[0], ys[1], nb=1),
         R.dot_cross(*[gpu(t) for t in xs + ys], nb=1))


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("shape", [(128, 100), (1, 37), (33, 1), (65, 97)])
def test_transpose2_matches_host(bits, shape):
    """k_transpose2 (32 x 32 LDS tiles, ragged edges) equals the host's transposes."""
    a0, a1 = rand_rt(shape, bits, 60), rand_rt(shape, bits, 61)
    h0, h1 = R.transpose2(a0, a1)
    d0, d1 = R.transpose2(gpu(a0), gpu(a1))
    same(h0, d0)
    same(h1, d1)
    same(h0, R.transpose(a0))


@pytest.mark.parametrize("bits", [64, 128])
def test_gemm_cross_matches_host(bits):
    M, K, N = 96, 160, 128
    xs = [rand_rt((3, M, K), bits, 20 + i) for i in range(2)]
    ys = [rand_rt((3, K, N), bits, 30 + i) for i in range(2)]
    h = R.dot_cross(xs[0], xs[1], ys[0], ys[1], nb=1)
    d = R.dot_cross(gpu(xs[0]), gpu(xs[1]), gpu(ys[0]), gpu(ys[1]), nb=1)
    same(h, d)


def test_gemm_mfma_asymmetric_identity():
    # A = I with an asymmetric B catches a transposed C write (guide §3)
    n = 64
    eye = R.from_ints([[1 if i == j else 0 for j in range(n)] for i in range(n)], 128, "cuda")
    vals = [[random.Random(i * n + j).getrandbits(128) for j in range(n)] for i in range(n)]
    b = R.from_ints(vals, 128, "cuda")
    nat.lib().mx_set_gemm_impl(2)
    try:
        c = R.dot(eye, b)
    finally:
        nat.lib().mx_set_gemm_impl(0)
    assert (R.to_ints(c) == R.to_ints(b)).all()


def test_gemm_long_k_split():
    bits = 128
    a, b = rand_rt((1, 64, 9000), bits, 40), rand_rt((1, 9000, 64), bits, 41)
    same(R.dot(a, b, nb=1), R.dot(gpu(a), gpu(b), nb=1))


def _const_limbs(digit, bits):
    """The ring element whose balanced base-256 limbs all equal ``digit``."""
    return sum(digit * 256**l for l in range(bits // 8)) % (1 << bits)


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("da,db", [(-128, -128), (-128, 127), (127, 127)])
def test_gemm_worst_case_limbs_at_max_k(bits, da, db):
    """Every limb at the extreme of [-128, 127] and K' at the largest unsplit chunk (8192
    for Z_2^128, 16384 for Z_2^64): the i32 diagonal accumulators of the MFMA kernels must
    stay exact (header of csrc/gemm_mfma.hip).  Every output equals K.a.b mod 2^bits."""
    K = 8192 if bits == 128 else 16384
    M, N = 64, 130  # N not a multiple of the 64x128 Z_2^64 block tile
    va, vb = _const_limbs(da, bits), _const_limbs(db, bits)
    a = R.from_ints([[va] * K] * M, bits, "cuda")
    b = R.from_ints([[vb] * N] * K, bits, "cuda")
    c = R.to_ints(R.dot(a, b))
    want = (K * va * vb) % (1 << bits)
    assert (c == want).all()


@pytest.mark.parametrize("bits", [64, 128])
def test_gemm_cross_long_k_split(bits):
    """Mode 1 (K-doubled RSS cross GEMM) with K' = 2K above the exact-chunk limit, so the
    host splits K and the kernel accumulates into C."""
    M, K, N = 64, 5000 if bits == 128 else 9000, 72
    xs = [rand_rt((1, M, K), bits, 50 + i) for i in range(2)]
    ys = [rand_rt((1, K, N), bits, 60 + i) for i in range(2)]
    h = R.dot_cross(xs[0], xs[1], ys[0], ys[1], nb=1)
    d = R.dot_cross(gpu(xs[0]), gpu(xs[1]), gpu(ys[0]), gpu(ys[1]), nb=1)
    same(h, d)


@pytest.mark.parametrize("bits", [64, 128])
def test_gemm_multi_tile_odd_ksteps(bits):
    """Several block tiles per batch, ragged M/N edges and an odd number of k-steps (the
    pipelined kernels unroll the k-loop by two)."""
    M, K, N = 200, 330, 260
    a, b = rand_rt((3, M, K), bits, 70), rand_rt((3, K, N), bits, 71)
    same(R.dot(a, b, nb=1), R.dot(gpu(a), gpu(b), nb=1))


@pytest.mark.parametrize("bits", [64, 128])
def test_fused_protocol_kernels_match_host(bits):
    from moose_amd.ir.computation import ReplicatedPlacement
    from moose_amd.protocols import replicated as rep
    from moose_amd.runtime.session import HV, StackedSession

    plc = ReplicatedPlacement(("a", "b", "c"))
    res = []
    for dev in ("cpu", "cuda"):
        s = StackedSession(dev, seed=9)
        x = HV("b", R.encode(torch.linspace(-20, 20, 4099, dtype=torch.float64).to(dev), 23, bits))
        X = rep.share(s, plc, x)
        T = rep.trunc_pr(s, rep.mul(s, X, X), 23)
        B = rep.bit_decompose(s, X)  # fused Kogge-Stone levels (k_ks_level3)
        res.append([t.cpu() for t in (X.s0.v.data, X.s1.v.data, T.s0.v.data, T.s1.v.data,
                                      B.s0.v.data, B.s1.v.data)])
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("both", [True, False])
def test_ks_cross1_matches_host(bits, both):
    """SPMD per-party Kogge-Stone level kernel (k_ks_cross1): GPU == CPU bitwise."""
    xs = [rand_rt((3, 37), bits, 60 + i) for i in range(4)]
    keys = (bytes(range(16)), bytes(range(16, 32)))
    cpu = R.ks_cross1(*xs, 3, both, keys, 11)
    dev = R.ks_cross1(*[gpu(x) for x in xs], 3, both, keys, 11)
    same(cpu, dev)


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("both", [True, False])
@pytest.mark.parametrize("n", [37, 3000])
def test_ks_cross1_slots_latency_form_matches_host(bits, both, n):
    """The key-slot Kogge-Stone level kernels of the per-party adders (ks_cross1_s and the
    xor-folding ks_cross1x_s; small launches take the latency form k_ks_cross1_lat):
    GPU == CPU bitwise, keys read from device / host key slots."""
    from moose_amd.runtime.keys import KeyTable

    xs = [rand_rt((n,), bits, 80 + i) for i in range(6)]
    raw = [bytes(range(16)), bytes(range(16, 32))]
    out = {}
    for dev in ("cpu", "cuda"):
        kt = KeyTable(dev, capacity=4)
        kt._write(0, raw)
        slots = [kt.ptr(0), kt.ptr(1)]
        ys = [x if dev == "cpu" else gpu(x) for x in xs]
        z = R.ks_cross1_s(*ys[:4], 5, both, slots, 23)
        zx, (go0, go1) = R.ks_cross1x_s(ys[0], ys[1], ys[4], ys[5], ys[2], ys[3], 3, both, slots,
                                        29)
        out[dev] = [t.data.cpu() for t in (z, zx, go0, go1)]
        torch.cuda.synchronize()
    for a, b in zip(out["cpu"], out["cuda"]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("bits", [64, 128])
def test_binary_slot_matches_host(bits):
    """Public operand on one share slot in one kernel (k_binary_slot): GPU == CPU."""
    a = rand_rt((3, 5, 7), bits, 70)
    for b in (rand_rt((5, 7), bits, 71), rand_rt((), bits, 72)):
        for which in (0, 2):
            same(R.binary_slot("add", a, b, which), R.binary_slot("add", gpu(a), gpu(b), which))


@pytest.mark.parametrize("bits", [64, 128])
def test_dot_zero_share_overlap_bitwise(bits, monkeypatch):
    """rep.dot with the zero-share keystream generated on a side stream during the GEMM
    (StackedSession.p_dot_zs_reshare) == the sequential fused path, bitwise."""
    from moose_amd.ir.computation import ReplicatedPlacement
    from moose_amd.protocols import replicated as rep
    from moose_amd.runtime.session import HV, StackedSession

    plc = ReplicatedPlacement(("a", "b", "c"))
    res = []
    g = torch.Generator(device="cpu").manual_seed(7)
    xf = torch.rand(1024, 96, dtype=torch.float64, generator=g).cuda()
    yf = torch.rand(96, 1024, dtype=torch.float64, generator=g).cuda()
    for flag in ("1", "0"):
        monkeypatch.setenv("MOOSEX_OVERLAP_ZS", flag)
        s = StackedSession("cuda", seed=3)
        x, y = R.encode(xf, 20, bits), R.encode(yf, 20, bits)
        X, Y = rep.share(s, plc, HV("a", x)), rep.share(s, plc, HV("b", y))
        Z = rep.dot(s, X, Y)
        res.append((Z.s0.v.data.cpu(), Z.s1.v.data.cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("kind", ["arith", "bool"])
def test_rss_cross_kp_matches_host(bits, kind):
    """Per-party key pairs (cyclic multi-GPU layout): device kernel == host kernel, and
    party p's zero share uses exactly keys 2p and 2p+1."""
    from moose_amd.runtime.keys import KeyTable

    keys = [bytes([7 * i + 1] * 16) for i in range(6)]
    tabs, alive = [], []  # keep both tables alive: the kernels read through raw pointers
    for dev in ("cpu", "cuda"):
        kt = KeyTable(dev)
        alive.append(kt)
        base = kt.alloc(6)
        kt._write(base, keys)
        tabs.append([kt.ptr(base + i) for i in range(6)])
    x0, x1 = rand_rt((3, 1000), bits, 11), rand_rt((3, 1000), bits, 12)
    y0, y1 = rand_rt((3, 1000), bits, 13), rand_rt((3, 1000), bits, 14)
    host = R.rss_cross_kp(kind, x0, x1, y0, y1, tabs[0], 99)
    dev = R.rss_cross_kp(kind, gpu(x0), gpu(x1), gpu(y0), gpu(y1), tabs[1], 99)
    same(host, dev)
    # party 1 alone with its own pair == the one-party generic kernel
    one = R.rss_cross(kind, R.RT(x0.data[1], bits), R.RT(x1.data[1], bits),
                      R.RT(y0.data[1], bits), R.RT(y1.data[1], bits), keys[2:4], 99, 1)
    assert torch.equal(one.data, host.data[1])


@pytest.mark.parametrize("bits", [64, 128])
def test_dot_cross_rows_prepared_b(bits):
    """Row blocks through the prepared-B GEMM (pipelined dot) == rows of the full product."""
    xs = [rand_rt((3, 300, 96), bits, 80 + i) for i in range(2)]
    ys = [rand_rt((3, 96, 80), bits, 90 + i) for i in range(2)]
    full = R.dot_cross(*xs, *ys, nb=1)
    g = [gpu(t) for t in xs + ys]
    pb = R.PreparedCross(g[2], g[3])
    assert pb.lb is not None
    for r0, r1 in ((0, 75), (75, 150), (150, 300)):
        part = R.dot_cross_rows(g[0], g[1], r0, r1, pb)
        assert torch.equal(part.data.cpu(), full.data[:, r0:r1])


def _slot_tables(n):
    from moose_amd.runtime.keys import KeyTable

    keys = [bytes([(13 * i + 5) % 256] * 16) for i in range(n)]
    tabs = []
    for dev in ("cpu", "cuda"):
        kt = KeyTable(dev)
        base = kt.alloc(n)
        kt._write(base, keys)
        tabs.append(kt)
    return tabs, [[t.ptr(base + i) for i in range(n)] for t in tabs]


@pytest.mark.parametrize("bits", [64, 128])
def test_trunc_party_rounds_match_host(bits):
    """Per-party TruncPr round kernels (cyclic layout): device == host for every output."""
    tabs, (hs, ds) = _slot_tables(6)  # tabs keeps both tables alive
    nonces = [11, 12, 13, 14, 15, 16]
    s0, s1 = rand_rt((3, 777), bits, 100), rand_rt((3, 777), bits, 101)
    h = R.trunc_party_r0(s0, s1, 23, [0, 1, 2], hs, nonces)
    d = R.trunc_party_r0(gpu(s0), gpu(s1), 23, [0, 1, 2], ds, nonces)
    assert torch.equal(h[0], d[0].cpu())  # every role's outgoing message
    for a, b in zip(h[1:], d[1:]):  # msg_rm and the new shares: the dealer's component only
        assert torch.equal(a[2], b[2].cpu())
    rmk, rrt = rand_rt((3, 777), bits, 102), rand_rt((3, 777), bits, 103)
    rrm = torch.randint(0, 2**62, (3, 777), dtype=torch.int64)
    out_h = [t.clone() for t in h[2:]]
    out_d = [t.clone() for t in d[2:]]
    wh = R.trunc_party_r1(h[0], rmk.data, rrt.data, rrm, *out_h, bits, 23, [0, 1, 2], hs, nonces)
    wd = R.trunc_party_r1(d[0], rmk.data.cuda(), rrt.data.cuda(), rrm.cuda(), *out_d, bits, 23,
                          [0, 1, 2], ds, nonces)
    assert torch.equal(wh[:2], wd.cpu()[:2])
    assert torch.equal(out_h[0][:1], out_d[0].cpu()[:1])
    assert torch.equal(out_h[1][1:2], out_d[1].cpu()[1:2])


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("j", [0, 1, 2])
def test_share_party_matches_host(bits, j):
    tabs, (hs, ds) = _slot_tables(6)
    x = rand_rt((500,), bits, 110 + j)
    rel = [(c - j) % 3 for c in range(3)]
    h = R.share_party("arith", x, 3, rel, hs, 21, 22)
    d = R.share_party("arith", gpu(x), 3, rel, ds, 21, 22)
    j1 = (j + 1) % 3
    assert torch.equal(h[1], d[1].cpu())
    keep = [c for c in range(3) if c != j1]  # the j+1 component's s0 arrives by message
    assert torch.equal(h[0][keep], d[0].cpu()[keep])
