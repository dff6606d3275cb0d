"""Host ring kernels vs python-int arithmetic (reference replicated/mod.rs:630-696
fuzz tests and host/ops.rs ring kernels)."""
import random

import numpy as np
import pytest
import torch
from hypothesis import given
from hypothesis import settings
from hypothesis import strategies as st

from moose_amd.ops import ring as R

MASK = {64: (1 << 64) - 1, 128: (1 << 128) - 1}


def test_aes_fips197_vector():
    key = bytes(range(16))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    assert R.aes_encrypt(key, pt).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def _chacha_block(key_words, consts, ctr_words, nonce_words, rounds):
    m = 0xFFFFFFFF
    st = list(consts) + list(key_words) + list(ctr_words) + list(nonce_words)
    x = list(st)

    def qr(a, b, c, d):
        for (p, q, r, k) in ((a, b, d, 16), (c, d, b, 12), (a, b, d, 8), (c, d, b, 7)):
            x[p] = (x[p] + x[q]) & m
            x[r] ^= x[p]
            x[r] = ((x[r] << k) | (x[r] >> (32 - k))) & m

    for _ in range(rounds // 2):
        qr(0, 4, 8, 12), qr(1, 5, 9, 13), qr(2, 6, 10, 14), qr(3, 7, 11, 15)
        qr(0, 5, 10, 15), qr(1, 6, 11, 12), qr(2, 7, 8, 13), qr(3, 4, 9, 14)
    return b"".join(((x[i] + st[i]) & m).to_bytes(4, "little") for i in range(16))


def test_chacha_core_rfc7539_vector():
    """The quarter-round / double-round structure against RFC 7539 section 2.3.2."""
    words = lambda b: [int.from_bytes(b[i:i + 4], "little") for i in range(0, len(b), 4)]  # noqa
    sigma = words(b"expand 32-byte k")
    out = _chacha_block(words(bytes(range(32))), sigma, [1],
                        words(bytes.fromhex("000000090000004a00000000")), 20)
    assert out[:16].hex() == "10f1e7e4d13b5915500fdd1fa32071c4"


def _prf_stream(key, nonce, nchunks):
    """moosex PRF (csrc/prf_core.h): ChaCha12, 128-bit key, 64-bit block counter and nonce;
    chunk c = 16-byte part (c >> 6) & 3 of block ((c >> 8) << 6) | (c & 63)."""
    words = lambda b: [int.from_bytes(b[i:i + 4], "little") for i in range(0, len(b), 4)]  # noqa
    tau = words(b"expand 16-byte k")
    kw = words(key) * 2
    out = []
    for c in range(nchunks):
        blk, part = ((c >> 8) << 6) | (c & 63), (c >> 6) & 3
        b = _chacha_block(kw, tau, [blk & 0xFFFFFFFF, blk >> 32],
                          [nonce & 0xFFFFFFFF, nonce >> 32], 12)
        out.append(b[16 * part:16 * part + 16])
    return b"".join(out)


def test_prg_is_the_chacha12_stream():
    key = bytes(range(16))
    ks = R.prg_bytes(key, 5, 300 * 16).numpy().tobytes()
    assert ks == _prf_stream(key, 5, 300)
    # offsets are consistent
    tail = R.prg_bytes(key, 5, 32, ctr0=2).numpy().tobytes()
    assert tail == ks[32:64]


def test_prf_expand_elements_follow_the_stream():
    key = bytes(range(3, 19))
    ref = _prf_stream(key, 77, 600)
    for bits, per in ((128, 1), (64, 2)):
        got = R.to_ints(R.prf_expand([key], 77, (700,), bits, "cpu"))[0]
        for i in (0, 1, 63, 64, 65, 255, 256, 299, 599 // per):
            c, j = divmod(i, per)
            chunk = ref[16 * c:16 * c + 16]
            want = int.from_bytes(chunk[8 * j:8 * j + bits // 8] if per == 2 else chunk, "little")
            assert int(got[i]) == want


@settings(max_examples=40, deadline=None)
@given(
    st.sampled_from([64, 128]),
    st.lists(st.integers(min_value=0), min_size=1, max_size=24),
    st.integers(min_value=0, max_value=2**20),
)
def test_fuzzy_elementwise(bits, vals, seed):
    rnd = random.Random(seed)
    xs = [v & MASK[bits] for v in vals]
    ys = [rnd.getrandbits(bits) for _ in xs]
    a, b = R.from_ints(xs, bits), R.from_ints(ys, bits)
    m = MASK[bits]
    for op, f in (("add", lambda p, q: p + q), ("sub", lambda p, q: p - q),
                  ("mul", lambda p, q: p * q), ("xor", lambda p, q: p ^ q),
                  ("and", lambda p, q: p & q), ("or", lambda p, q: p | q)):
        assert list(R.to_ints(R.binary(op, a, b))) == [f(p, q) & m for p, q in zip(xs, ys)]
    k = rnd.randrange(bits)
    assert list(R.to_ints(a.shl(k))) == [(p << k) & m for p in xs]
    assert list(R.to_ints(a.shr(k))) == [p >> k for p in xs]
    assert list(R.to_ints(-a)) == [(-p) & m for p in xs]


@pytest.mark.parametrize("bits", [64, 128])
def test_fuzzy_dot(bits):
    rnd = random.Random(bits)
    for (m, k, n) in [(1, 1, 1), (3, 5, 4), (7, 1, 9), (2, 24, 3)]:
        A = [[rnd.getrandbits(bits) for _ in range(k)] for _ in range(m)]
        B = [[rnd.getrandbits(bits) for _ in range(n)] for _ in range(k)]
        C = R.to_ints(R.dot(R.from_ints(A, bits), R.from_ints(B, bits)))
        for i in range(m):
            for j in range(n):
                assert C[i][j] == sum(A[i][t] * B[t][j] for t in range(k)) & MASK[bits]


@pytest.mark.parametrize("bits", [64, 128])
def test_dot_cross_equals_three_products(bits):
    rnd = random.Random(7)
    mk = lambda r, c: R.from_ints([[rnd.getrandbits(bits) for _ in range(c)] for _ in range(r)], bits)
    x0, x1, y0, y1 = mk(4, 6), mk(4, 6), mk(6, 5), mk(6, 5)
    got = R.dot_cross(x0, x1, y0, y1)
    want = R.dot(x0, y0) + R.dot(x0, y1) + R.dot(x1, y0)
    assert (R.to_ints(got) == R.to_ints(want)).all()


@pytest.mark.parametrize("bits", [64, 128])
def test_vector_matrix_shapes(bits):
    v = R.from_ints([1, 2, 3], bits)
    m = R.from_ints([[1, 0], [0, 1], [1, 1]], bits)
    assert list(R.to_ints(R.dot(v, m))) == [4, 5]
    assert int(R.to_ints(R.dot(v, v))) == 14
    mt = R.from_ints([[1, 0, 1], [0, 1, 1]], bits)
    assert list(R.to_ints(R.dot(mt, v))) == [4, 5]


@pytest.mark.parametrize("bits", [64, 128])
def test_encode_decode_truncates_like_reference(bits):
    x = torch.tensor([1.5, -2.25, 3.0, -1e-9, 123.456], dtype=torch.float64)
    e = R.encode(x, 23, bits)
    si = R.to_signed_ints(e)
    assert list(si) == [int(v * 2**23) for v in x.tolist()]  # truncation toward zero
    d = R.decode(e, 23)
    assert torch.allclose(d, x, atol=2**-22)


@pytest.mark.parametrize("bits", [64, 128])
def test_sum_and_compare(bits):
    a = R.from_ints([[1, 2, 3], [4, 5, 6]], bits)
    assert list(R.to_ints(R.sum(a, 0))) == [5, 7, 9]
    assert list(R.to_ints(R.sum(a, 1))) == [6, 15]
    assert int(R.to_ints(R.sum(a, None))) == 21
    neg = R.from_ints([(-3) & MASK[bits], 2], bits)
    pos = R.from_ints([1, 5], bits)
    assert R.compare("lt", neg, pos).data.tolist() == [1, 1]
    assert R.compare("msb", neg).data.tolist() == [1, 0]


@pytest.mark.parametrize("bits", [1, 64, 128])
def test_zero_share_sums_to_zero(bits):
    keys = [bytes([i]) * 16 for i in range(3)]
    kind = "bool" if bits == 1 else "arith"
    z = R.zero_share(kind, (3, 50), bits, keys + keys[:1], 11, 3, "cpu")
    v = R.to_ints(z)
    if kind == "bool":
        assert ((v[0] ^ v[1] ^ v[2]) == 0).all()
    else:
        assert (((v[0] + v[1] + v[2]) & MASK[bits]) == 0).all()


def test_bit_extract_inject():
    x = R.from_ints([5, (1 << 127) + 2], 128)
    assert R.bit_extract(x, 0).data.tolist() == [1, 0]
    assert R.bit_extract(x, 127).data.tolist() == [0, 1]
    b = R.RT(torch.tensor([1, 0], dtype=torch.uint8), 1)
    assert list(R.to_ints(R.ring_inject(b, 100, 128))) == [1 << 100, 0]
    assert list(R.to_ints(R.ring_inject(b, 3, 64))) == [8, 0]


def test_cast_between_rings():
    x = R.from_ints([(1 << 100) + 7, 3], 128)
    assert list(R.to_ints(R.cast(x, 64))) == [7, 3]
    y = R.from_ints([MASK[64], 1], 64)
    assert list(R.to_ints(R.sign_extend(y, 64, 128))) == [MASK[128], 1]


def test_from_to_ints_roundtrip():
    vals = np.array([[0, 1], [MASK[128], 1 << 64]], dtype=object)
    assert (R.to_ints(R.from_ints(vals, 128)) == vals).all()
