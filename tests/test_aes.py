"""AES: generated Bristol circuit vs AES-NI, host and replicated AES-GCM decryption
(reference ``bristol_fashion`` + ``encrypted`` tests; FIPS-197 appendix C.1 vector)."""
import os

import numpy as np
import pytest
import torch

import moose_amd as pm
from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ops import ring as R
from moose_amd.protocols import aes
from moose_amd.protocols import replicated as rep
from moose_amd.protocols.aes_circuit import aes128_circuit
from moose_amd.protocols.bristol import LevelledCircuit
from moose_amd.protocols.bristol import parse_bristol
from moose_amd.runtime.local import LocalMooseRuntime
from moose_amd.runtime.session import HV
from moose_amd.runtime.session import StackedSession


def _bits(b: bytes):
    return [(b[i // 8] >> (7 - i % 8)) & 1 for i in range(8 * len(b))]


def _bytes(bits):
    return bytes(sum(int(bits[8 * j + k]) << (7 - k) for k in range(8)) for j in range(len(bits) // 8))


def test_circuit_matches_fips197_and_aesni():
    lc = aes.levelled_aes()
    assert lc.depth == 60  # 10 S-box layers of AND depth 6 (key schedule alongside)
    keys = [bytes.fromhex("000102030405060708090a0b0c0d0e0f")] + [os.urandom(16) for _ in range(3)]
    blocks = [bytes.fromhex("00112233445566778899aabbccddeeff")] + [os.urandom(16) for _ in range(3)]
    inp = torch.tensor([_bits(k) + _bits(b) for k, b in zip(keys, blocks)], dtype=torch.uint8).T
    out = lc.eval_plain(inp)
    got = [_bytes(out[:, i].tolist()) for i in range(len(keys))]
    assert got[0].hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"
    assert got == [R.aes_encrypt(k, b) for k, b in zip(keys, blocks)]


def test_bristol_text_roundtrip():
    c = aes128_circuit()
    c2 = parse_bristol(c.to_bristol())
    assert c2.num_wires == c.num_wires and c2.stats() == c.stats()
    assert c.stats()["AND"] == 6400  # as the reference's bristol_fashion/aes_128.txt


def test_sbox_circuit_all_inputs():
    """The 32-AND S-box sub-circuit against the FIPS-197 S-box table, all 256 bytes."""
    from moose_amd.protocols.aes_circuit import _Builder
    from moose_amd.protocols.bristol import Circuit

    b = _Builder(8)
    outs = b.sbox(list(range(8)))  # lsb-first byte in, lsb-first byte out
    assert sum(g.op == "AND" for g in b.gates) == 32
    outs = [b.copy(w) for w in outs]
    circ = Circuit(b.n, [8], [8], b.gates)
    inp = torch.tensor([[(v >> i) & 1 for i in range(8)] for v in range(256)],
                       dtype=torch.uint8).T
    from moose_amd.protocols.bristol import LevelledCircuit

    got = LevelledCircuit(circ).eval_plain(inp)
    sbox = _sbox_table()
    for v in range(256):
        assert sum(int(got[i, v]) << i for i in range(8)) == sbox[v], v


def _sbox_table():
    def mul(a, b):
        r = 0
        while b:
            if b & 1:
                r ^= a
            a <<= 1
            if a & 0x100:
                a ^= 0x11B
            b >>= 1
        return r

    inv = [0] + [next(b for b in range(1, 256) if mul(a, b) == 1) for a in range(1, 256)]
    out = []
    for a in range(256):
        x, s = inv[a], inv[a]
        for i in range(1, 5):
            s ^= ((x << i) | (x >> (8 - i))) & 0xFF
        out.append(s ^ 0x63)
    return out


def test_small_bristol_circuit_levelling():
    # (a AND b) XOR (NOT c), then AND with a: depth 2
    text = "4 7\n2 1 2\n1 1\n\n2 1 0 1 3 AND\n1 1 2 4 INV\n2 1 3 4 5 XOR\n2 1 5 0 6 AND\n"
    lc = LevelledCircuit(parse_bristol(text))
    assert lc.depth == 2
    for a in (0, 1):
        for b in (0, 1):
            for c in (0, 1):
                out = lc.eval_plain(torch.tensor([[a], [b], [c]], dtype=torch.uint8))
                assert int(out[0, 0]) == (((a & b) ^ (1 - c)) & a)


def test_host_and_replicated_decrypt():
    key = os.urandom(16)
    vals = np.array([1.5, -2.25, 1000.125])
    ct = aes.encrypt_fixed(key, vals, 40)
    kbits = np.array(_bits(key), dtype=np.uint8)
    pt = aes.host_decrypt(kbits, ct)
    np.testing.assert_allclose(R.decode(pt, 40).numpy(), vals)
    sess = StackedSession("cpu", seed=3)
    plc = ReplicatedPlacement(("a", "b", "c"))
    K = rep.share(sess, plc, HV("a", R.RT(torch.as_tensor(kbits), 1)), kind="bool")
    C = rep.share(sess, plc, HV("b", R.RT(torch.as_tensor(ct), 1)), kind="bool")
    T = aes.rep_decrypt(sess, plc, K, C)
    np.testing.assert_allclose(R.decode(rep.reveal(sess, T, "c").v, 40).numpy(), vals)


@pytest.mark.parametrize("host_decrypt", [True, False])
def test_decrypt_computation(host_decrypt):
    alice, bob, carole = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
    rp = pm.replicated_placement("rep", players=[alice, bob, carole])
    dec = alice if host_decrypt else rp

    @pm.computation
    def f(key: pm.Argument(rp, vtype=pm.AesKeyType()),
          ct: pm.Argument(alice, vtype=pm.AesTensorType(pm.fixed(24, 40)))):
        with dec:
            data = pm.decrypt(key, ct)
        with alice:
            return pm.cast(data, pm.float64)

    key = os.urandom(16)
    kb = np.array(_bits(key), dtype=np.bool_)
    s0 = np.random.default_rng(1).integers(0, 2, 128).astype(np.bool_)
    s1 = np.random.default_rng(2).integers(0, 2, 128).astype(np.bool_)
    s2 = kb ^ s0 ^ s1
    vals = np.array([[3.25, -7.5]])
    args = {"key/alice/share0": s0, "key/alice/share1": s1, "key/bob/share1": s1,
            "key/bob/share2": s2, "key/carole/share2": s2, "key/carole/share0": s0,
            "ct": aes.encrypt_fixed(key, vals, 40).astype(np.bool_)}
    out = LocalMooseRuntime(["alice", "bob", "carole"], device="cpu").evaluate_computation(f, args)
    np.testing.assert_allclose(list(out.values())[0], vals)
