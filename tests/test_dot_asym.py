"""Asymmetric local products of a replicated matrix product (ops/ring.py dot_cross_asym,
csrc/gemm_crt.hip run_crt_asym): z_0 = (a + b)(c + d), z_1 = b (c + d) + a d,
z_2 = a d + b c for party p's shares (a, b) of x and (c, d) of y.

CPU: each z_p equals its formula evaluated with plain ring products, the three sum to the
symmetric form's sum (= x.y), and a stacked session's fixed-point product through them
matches float64.  GPU: the one-launch CRT form (rolled and two-stack) is bitwise the generic
form, and a device session's shares equal a CPU session's bit for bit."""
import pytest
import torch

from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ops import ring as R
from moose_amd.protocols import replicated as rep
from moose_amd.runtime.session import HV
from moose_amd.runtime.session import StackedSession

PLC = ReplicatedPlacement(("a", "b", "c"))


def _rand(shape, bits, seed):
    g = torch.Generator().manual_seed(seed)
    return R.RT(torch.randint(-(2**63), 2**63 - 1, shape + ((2,) if bits == 128 else ()),
                              generator=g, dtype=torch.int64), bits)


def _at(t, p):
    return R.RT(t.data[p], t.bits)


def _same(a, b):
    assert a.bits == b.bits
    assert torch.equal(a.data.cpu(), b.data.cpu())


def _formula(x0, x1, y0, y1):
    add = lambda u, v: R.binary("add", u, v)  # noqa: E731
    out = []
    for p in range(3):
        a, b, c, d = (_at(t, p) for t in (x0, x1, y0, y1))
        if p == 0:
            out.append(R.dot(add(a, b), add(c, d)))
        elif p == 1:
            out.append(add(R.dot(b, add(c, d)), R.dot(a, d)))
        else:
            out.append(add(R.dot(a, d), R.dot(b, c)))
    return out


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("mkn", [(3, 5, 4), (17, 33, 9)])
def test_asym_products_formula_and_sum(bits, mkn):
    M, K, N = mkn
    x0, y0 = _rand((3, M, K), bits, 1), _rand((3, K, N), bits, 2)
    x1 = R.RT(torch.roll(x0.data, -1, dims=0), bits)
    y1 = R.RT(torch.roll(y0.data, -1, dims=0), bits)
    z = R.dot_cross_asym(x0, x1, y0, y1)
    for p, want in enumerate(_formula(x0, x1, y0, y1)):
        _same(_at(z, p), want)
    sym = R.dot_cross(x0, x1, y0, y1, nb=1)
    total = lambda t: R.binary("add", R.binary("add", _at(t, 0), _at(t, 1)), _at(t, 2))  # noqa: E731
    _same(total(z), total(sym))
    # the rolled call (second stacks implied) is the same
    _same(R.dot_cross_asym(x0, None, y0, None, rolled=True), z)


def _session_dot(device, n, bits=128, seed=5):
    g = torch.Generator().manual_seed(n)
    xa = torch.rand(n, n, generator=g, dtype=torch.float64) * 4 - 2
    ya = torch.rand(n, n, generator=g, dtype=torch.float64) * 4 - 2
    s = StackedSession(device, seed=seed)
    enc = lambda t: R.encode(t.to(device), 23, bits)  # noqa: E731
    X = rep.share(s, PLC, HV("a", enc(xa)))
    Y = rep.share(s, PLC, HV("b", enc(ya)))
    Z = rep.dot_trunc(s, X, Y, 23)
    out = R.decode(R.RT(rep.reveal(s, Z, "c").v.data, bits), 23)
    return Z, out.cpu(), xa @ ya


def test_session_dot_uses_asym_and_matches_float():
    from moose_amd.runtime import session as S

    x = _rand((3, 256, 256), 128, 3)
    assert S._asym_applies(x, x) and not S._asym_applies(_rand((3, 255, 256), 128, 3), x)
    _, out, want = _session_dot("cpu", 256)
    assert (out - want).abs().max() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("mkn", [(256, 256, 256), (300, 512, 270), (260, 300, 256)])
def test_gpu_asym_one_launch_matches_generic(bits, mkn):
    """mx_gemm_asym (rolled: x1/y1 implied; and with explicit second stacks) == the generic
    form on the CPU, bitwise; K not a multiple of 64 takes the generic device form."""
    M, K, N = mkn
    x0, y0 = _rand((3, M, K), bits, 11), _rand((3, K, N), bits, 12)
    x1r = R.RT(torch.roll(x0.data, -1, dims=0).contiguous(), bits)
    y1r = R.RT(torch.roll(y0.data, -1, dims=0).contiguous(), bits)
    want = R.dot_cross_asym(x0, x1r, y0, y1r)
    g = lambda t: R.RT(t.data.cuda(), t.bits)  # noqa: E731
    _same(R.dot_cross_asym(g(x0), None, g(y0), None, rolled=True), want)
    # unrelated second stacks (the cyclic layout's components)
    x1, y1 = _rand((3, M, K), bits, 13), _rand((3, K, N), bits, 14)
    _same(R.dot_cross_asym(g(x0), g(x1), g(y0), g(y1)), R.dot_cross_asym(x0, x1, y0, y1))


@pytest.mark.gpu
def test_gpu_session_dot_asym_bitwise_cpu():
    """A device stacked session's product shares (asymmetric CRT GEMM + fused tail) equal a
    CPU session's (generic asymmetric products + generic tail) bit for bit."""
    zg, og, want = _session_dot("cuda:0", 320)
    zc, oc, _ = _session_dot("cpu", 320)
    assert torch.equal(zg.s0.v.data.cpu(), zc.s0.v.data)
    assert torch.equal(zg.s1.v.data.cpu(), zc.s1.v.data)
    assert torch.equal(og, oc)
    assert (og - want).abs().max() < 1e-4


def _cyclic_vs_stacked(device):
    from moose_amd.parallel.cyclic import CyclicSession
    from moose_amd.parallel.cyclic import RingComm

    cyc = CyclicSession(RingComm(0, 1, device), {"a": 0, "b": 1, "c": 2}, device, seed=9,
                        pipeline_chunks=1)
    keys = cyc.session_keys(PLC, 0)
    st = StackedSession("cpu", seed=9)
    st.fused = False
    st.keytable._write(st.setup(PLC), keys)
    res = []
    for sess, dev in ((cyc, device), (st, "cpu")):
        g = torch.Generator().manual_seed(4)
        a, b = (torch.rand(256, 256, generator=g, dtype=torch.float64) - 0.5 for _ in range(2))
        X = rep.share(sess, PLC, HV("a", R.encode(a.to(dev), 23, 128)))
        Y = rep.share(sess, PLC, HV("b", R.encode(b.to(dev), 23, 128)))
        Z = rep.dot_trunc(sess, X, Y, 23)
        out = R.decode(R.RT(rep.reveal(sess, Z, "c").v.data, 128), 23).cpu()
        res.append((Z.s0.v.data.cpu(), Z.s1.v.data.cpu(), out, a @ b))
    (c0, c1, co, want), (s0, s1, so, _) = res
    assert torch.equal(c0, s0) and torch.equal(c1, s1) and torch.equal(co, so)
    assert (co - want).abs().max() < 1e-4


def test_cyclic_session_asym_bitwise_stacked():
    """The cyclic layout's session (components of different sessions: the two-stack form)
    takes the same asymmetric products as a stacked session: bitwise the same shares."""
    _cyclic_vs_stacked("cpu")


@pytest.mark.gpu
def test_gpu_cyclic_session_asym_bitwise_cpu_stacked():
    """On the device the cyclic session runs the one-launch five-image form (no roll)."""
    _cyclic_vs_stacked("cuda:0")
