"""Share-pair elementwise kernels (mx_ew_binary2 / mx_ew_unary2 / mx_ew_binary_slot2: both
replicated share vectors of a share-wise op in one launch) and the TruncPr kernel writing
into row views (mx_trunc_pr3_ko) agree exactly with the one-operand forms."""
import numpy as np
import pytest
import torch

from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ops import ring as R
from moose_amd.protocols import replicated as rep
from moose_amd.runtime.session import PV
from moose_amd.runtime.session import StackedSession

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _rand(shape, bits, dev, seed):
    rng = np.random.default_rng(seed)
    vals = rng.integers(0, 2**62, size=int(np.prod(shape)), dtype=np.int64).astype(object)
    vals = vals * (1 << (bits - 62)) + rng.integers(0, 2**40, size=vals.shape[0]).astype(object)
    return R.reshape(R.from_ints(vals % (1 << bits), bits, dev), shape)


def _eq(a, b):
    np.testing.assert_array_equal(R.to_ints(a), R.to_ints(b))


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("op", ["add", "sub", "mul", "xor", "and"])
def test_binary2_matches_binary(dev, bits, op):
    a0, b0, a1, b1 = (_rand((3, 37), bits, dev, s) for s in range(4))
    o0, o1 = R.binary2(op, a0, b0, a1, b1)
    _eq(o0, R.binary(op, a0, b0))
    _eq(o1, R.binary(op, a1, b1))
    c = _rand((1,), bits, dev, 9)  # scalar broadcast
    o0, o1 = R.binary2(op, a0, c, a1, c)
    _eq(o0, R.binary(op, a0, c))
    _eq(o1, R.binary(op, a1, c))


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("shape", [(128, 100), (1, 37), (65, 97)])
def test_transpose2_matches_transpose(dev, bits, shape):
    a0, a1 = _rand(shape, bits, dev, 5), _rand(shape, bits, dev, 6)
    o0, o1 = R.transpose2(a0, a1)
    _eq(o0, R.transpose(a0))
    _eq(o1, R.transpose(a1))


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("bits", [64, 128])
def test_unary2_and_slot2(dev, bits):
    a0, a1 = _rand((3, 5, 7), bits, dev, 1), _rand((3, 5, 7), bits, dev, 2)
    for op, k in (("neg", 0), ("shl", 5)):
        o0, o1 = R.unary2(op, a0, a1, k)
        _eq(o0, R.unary(op, a0, k))
        _eq(o1, R.unary(op, a1, k))
    c = _rand((5, 7), bits, dev, 3)
    o0, o1 = R.binary_slot2("add", a0, a1, c, 0, 2)
    _eq(o0, R.binary_slot("add", a0, c, 0))
    _eq(o1, R.binary_slot("add", a1, c, 2))


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("bits", [64, 128])
def test_trunc_into_row_views(dev, bits):
    """fused_trunc_pr(out=row views) writes the same shares as the dense form."""
    plc = ReplicatedPlacement(("alice", "bob", "carole"))
    shp = (3, 2, 11)
    x0, x1 = _rand(shp, bits, dev, 4), _rand(shp, bits, dev, 5)
    x = rep.RepTensor(plc, bits, "arith", PV(plc, x0), PV(plc, x1))
    nonces = (11, 12, 13, 14, 15, 16)
    s = StackedSession(dev, seed=7)
    d0, d1 = s.fused_trunc_pr(x, 20, nonces)
    big0 = R.zeros((3, 5, 11), bits, dev).data
    big1 = torch.zeros_like(big0)
    v0, v1 = PV(plc, R.RT(big0[:, 2:4], bits)), PV(plc, R.RT(big1[:, 2:4], bits))
    s.fused_trunc_pr(x, 20, nonces, out=(v0, v1))
    _eq(R.RT(big0[:, 2:4].contiguous(), bits), d0.v)
    _eq(R.RT(big1[:, 2:4].contiguous(), bits), d1.v)
    # rows outside the view are untouched
    assert not big0[:, :2].any() and not big0[:, 4:].any()


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("bits", [64, 128])
def test_slot_place2(dev, bits):
    x0, x1 = _rand((4, 3), bits, dev, 6), _rand((4, 3), bits, dev, 7)
    o0, o1 = R.slot_place2(x0, x1, 2, 1)
    z = np.zeros((4, 3), dtype=object)
    np.testing.assert_array_equal(R.to_ints(o0), np.stack([z, z, R.to_ints(x0)]))
    np.testing.assert_array_equal(R.to_ints(o1), np.stack([z, R.to_ints(x1), z]))


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("bits", [64, 128])
def test_slot_ops_broadcast_trailing_vector(dev, bits):
    """A public operand shaped like the slot's trailing axes repeats with that period."""
    a0, a1 = _rand((3, 5, 4), bits, dev, 8), _rand((3, 5, 4), bits, dev, 9)
    c = _rand((4,), bits, dev, 10)
    full = R.RT(c.data.unsqueeze(0).expand((5,) + tuple(c.data.shape)).contiguous(), bits)
    _eq(R.binary_slot("add", a0, c, 1), R.binary_slot("add", a0, full, 1))
    o0, o1 = R.binary_slot2("sub", a0, a1, c, 0, 2)
    _eq(o0, R.binary_slot("sub", a0, full, 0))
    _eq(o1, R.binary_slot("sub", a1, full, 2))


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("layout", ["dense", "views"])
@pytest.mark.parametrize("cols", [50, 3000])
def test_mul_trunc_fused_matches_two_steps(bits, layout, cols):
    """rep.mul_trunc's single kernel (mx_mul_trunc3_kv; latency form, and the throughput
    form at 18000 elements per party) produces exactly the shares of rep.mul followed by
    rep.trunc_pr (same keys, same nonce order)."""
    plc = ReplicatedPlacement(("alice", "bob", "carole"))
    shp = (3, 6, cols)
    xs = [_rand(shp, bits, "cuda", s) for s in (21, 22)]
    ys = [_rand(shp, bits, "cuda", s) for s in (23, 24)]
    if layout == "views":  # row slices of larger stacks, read in place
        xs = [R.RT(R.zeros((3, 9, cols), bits, "cuda").data, bits) for _ in range(2)]
        for i, s in enumerate((21, 22)):
            xs[i].data[:, 2:8] = _rand(shp, bits, "cuda", s).data
        xs = [R.RT(x.data[:, 2:8], bits) for x in xs]
    X = rep.RepTensor(plc, bits, "arith", PV(plc, xs[0]), PV(plc, xs[1]))
    Y = rep.RepTensor(plc, bits, "arith", PV(plc, ys[0]), PV(plc, ys[1]))
    s1, s2 = StackedSession("cuda", seed=3), StackedSession("cuda", seed=3)
    a = rep.mul_trunc(s1, X, Y, 20)
    b = rep.trunc_pr(s2, rep.mul(s2, X, Y), 20)
    _eq(a.s0.v, b.s0.v)
    _eq(a.s1.v, b.s1.v)


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("bits", [64, 128])
def test_lincomb2_matches_composition(dev, bits):
    a = [_rand((3, 4, 5), bits, dev, s) for s in range(31, 37)]
    c = _rand((5,), bits, dev, 40)
    o0, o1 = R.lincomb2([(1, a[0], a[1]), (1, a[2], a[3]), (-2, a[4], a[5])], c, 0, 2)
    for o, (x, y, z), w in ((o0, (a[0], a[2], a[4]), 0), (o1, (a[1], a[3], a[5]), 2)):
        want = R.binary("sub", R.binary("add", x, y), R.unary("shl", z, 1))
        _eq(o, R.binary_slot("add", want, c, w))
    o0, o1 = R.lincomb2([(-1, a[0], a[1])])
    _eq(o0, R.unary("neg", a[0]))
    _eq(o1, R.unary("neg", a[1]))


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("bits", [64, 128])
def test_sum_views2_of_one_stack(dev, bits):
    """AddN over the entries of a party-stacked batch reads them in place (mx_sum_views2)."""
    b0, b1 = _rand((3, 7, 4, 5), bits, dev, 50), _rand((3, 7, 4, 5), bits, dev, 51)
    v0 = [R.index_axis(b0, 0, i, nb=1) for i in range(7)]
    v1 = [R.index_axis(b1, 0, i, nb=1) for i in range(7)]
    assert not v0[1].data.is_contiguous()  # views, not copies
    o0, o1 = R.sum_views2(v0, v1)
    w0, w1 = v0[0], v1[0]
    for i in range(1, 7):
        w0, w1 = R.binary("add", w0, v0[i]), R.binary("add", w1, v1[i])
    _eq(o0, w0)
    _eq(o1, w1)
    assert R.sum_views2([v0[0], v0[2]], [v1[0], v1[1]]) is not None  # any even spacing
    assert R.sum_views2([v0[0], v0[1], v0[3]], v1[:3]) is None  # uneven: declined


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("bits", [64, 128])
def test_mul_public_trunc_matches_two_steps(dev, bits):
    """TruncPr with the public scalar folded in equals mul_public then trunc_pr."""
    plc = ReplicatedPlacement(("alice", "bob", "carole"))
    x0, x1 = _rand((3, 9, 7), bits, dev, 60), _rand((3, 9, 7), bits, dev, 61)
    X = rep.RepTensor(plc, bits, "arith", PV(plc, x0), PV(plc, x1))
    cv = (1 << (bits - 3)) + 12345
    c = R.fill((), cv, bits, dev)
    s1, s2 = StackedSession(dev, seed=5), StackedSession(dev, seed=5)
    a = rep.mul_public_trunc(s1, X, c, 20, value=cv)
    b = rep.trunc_pr(s2, rep.mul_public(s2, X, c), 20)
    _eq(a.s0.v, b.s0.v)
    _eq(a.s1.v, b.s1.v)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("mnk", [(6, 9, 5), (150, 40, 160)])
def test_dot_tail_fused_matches_two_steps(bits, mnk, monkeypatch):
    """rep.dot_trunc's one-kernel tail (zero share + reshare + TruncPr of the GEMM output,
    mx_mul_trunc3_kv with the product given; latency and throughput kernels) gives exactly
    the shares of rep.dot followed by rep.trunc_pr."""
    plc = ReplicatedPlacement(("alice", "bob", "carole"))
    M, K, N = mnk
    x0 = _rand((3, M, K), bits, "cuda", 61)
    y0 = _rand((3, K, N), bits, "cuda", 62)
    roll = lambda t: R.RT(torch.roll(t.data, -1, dims=0).contiguous(), bits)  # noqa: E731
    X = rep.RepTensor(plc, bits, "arith", PV(plc, x0), PV(plc, roll(x0)))
    Y = rep.RepTensor(plc, bits, "arith", PV(plc, y0), PV(plc, roll(y0)))
    s1, s2 = StackedSession("cuda", seed=5), StackedSession("cuda", seed=5)
    a = rep.dot_trunc(s1, X, Y, 20)
    monkeypatch.setenv("MOOSEX_DOT_TAIL", "0")
    b = rep.dot_trunc(s2, X, Y, 20)
    _eq(a.s0.v, b.s0.v)
    _eq(a.s1.v, b.s1.v)
    # the unfused pair is a valid sharing: s1 is s0 rolled by one party
    _eq(roll(a.s0.v), a.s1.v)


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("bits", [64, 128])
def test_share_pair_ring_buffer(dev, bits):
    """Share and TruncPr outputs of a stacked session are views of one 4-slot ring buffer
    (s1 = s0 rolled by one party, no second copy), and hold the same shares as two separate
    buffers (MOOSEX_RING4=0 path: R.empty2)."""
    plc = ReplicatedPlacement(("alice", "bob", "carole"))
    x0 = _rand((3, 4, 9), bits, dev, 70)
    roll = lambda t: R.RT(torch.roll(t.data, -1, dims=0).contiguous(), bits)  # noqa: E731
    X = rep.RepTensor(plc, bits, "arith", PV(plc, x0), PV(plc, roll(x0)))
    s = StackedSession(dev, seed=9)
    t0, t1 = s.fused_trunc_pr(X, 20, (1, 2, 3, 4, 5, 6))
    el = t0.v.data.element_size() * t0.v.data[0].numel()
    assert t1.v.data.data_ptr() - t0.v.data.data_ptr() == el  # one buffer, offset one slot
    _eq(roll(t0.v), t1.v)
    a, b = R.ring4((3, 5), bits, dev)
    assert b.data.data_ptr() - a.data.data_ptr() == a.data[0].numel() * a.data.element_size()
    R._RING4 = False
    try:
        u0, u1 = s.fused_trunc_pr(X, 20, (1, 2, 3, 4, 5, 6))
    finally:
        R._RING4 = True
    _eq(u0.v, t0.v)
    _eq(u1.v, t1.v)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("shapes", [((200, 10), (10, 2)), ((200, 10), (10,)), ((10,), (10, 3)),
                                    ((300, 96), (96, 80))])
def test_dot_public_pair_one_launch(bits, shapes):
    """rep.dot_public on a share-pair ring buffer: one product of the buffer's four slots
    with the public operand read in place (small: the VALU kernel, large: the strided
    GEMM); bitwise the per-share products, and the result is again a ring buffer."""
    xs, cs = shapes
    buf = _rand((4,) + xs, bits, "cuda", 1)
    buf.data[3].copy_(buf.data[0])  # ring buffer: slot 3 = slot 0
    s0, s1 = R.RT(buf.data[0:3], bits), R.RT(buf.data[1:4], bits)
    c = _rand(cs, bits, "cuda", 2)
    sess = StackedSession("cuda", seed=1)
    r = sess.p_dot_public_pair(None, PV(None, s0), PV(None, s1), type("P", (), {"v": c})())
    assert r is not None
    want0 = R.dot(s0, R.RT(c.data.unsqueeze(0).expand((3,) + tuple(c.data.shape)).contiguous(),
                           bits), nb=1)
    want1 = R.dot(s1, R.RT(c.data.unsqueeze(0).expand((3,) + tuple(c.data.shape)).contiguous(),
                           bits), nb=1)
    _eq(r[0].v, want0)
    _eq(r[1].v, want1)
    assert r[1].v.data.data_ptr() - r[0].v.data.data_ptr() == \
        r[0].v.data.stride(0) * r[0].v.data.element_size()


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
def test_b2a_prep_kernel_matches_generic(bits):
    """rep.b2a with its local steps in one kernel (StackedSession.p_b2a_prep) gives bitwise
    the shares of the generic Xor / RingInject / slot-placement steps (same seed)."""
    from moose_amd.runtime.session import HV

    plc = ReplicatedPlacement(owners=("a", "b", "c"))
    outs = []
    for fused in (True, False):
        sess = StackedSession("cuda", seed=7)
        sess.p_b2a = lambda *a, **k: None
        if not fused:
            sess.p_b2a_prep = lambda *a, **k: None
        x = rep.share(sess, plc, HV("a", _rand((300,), bits, "cuda", 3)))
        b = rep.msb(sess, x)
        y = rep.b2a(sess, b, bits)
        outs.append((y.s0.v, y.s1.v))
    _eq(outs[0][0], outs[1][0])
    _eq(outs[0][1], outs[1][1])


@pytest.mark.gpu
@pytest.mark.parametrize("bits,n,mirror", [(64, 301, False), (128, 300, False),
                                           (128, 300, True), (64, 70001, False),
                                           (128, 70001, True)])
def test_b2a_one_kernel_matches_generic(bits, n, mirror):
    """The whole of rep.b2a in one kernel (StackedSession.p_b2a, k_b2a3) gives bitwise the
    shares, the nonce position and the traffic records of the share + mul + lincomb steps
    (same seed; both share directions; latency and grid-stride sizes)."""
    from moose_amd.runtime.session import HV

    plc = ReplicatedPlacement(owners=("a", "b", "c"))
    outs = []
    for whole in (True, False):
        sess = StackedSession("cuda", seed=11)
        if mirror:
            sess.share_dirs = {"a": 2}
        if not whole:
            sess.p_b2a = lambda *a, **k: None
        xv = _rand((n,), bits, "cuda", 4)
        x = rep.share(sess, plc, HV("a", xv))
        y = rep.b2a(sess, rep.msb(sess, x), bits)
        nxt = rep.share(sess, plc, HV("b", _rand((7,), bits, "cuda", 5)))  # next nonce
        opened = rep.reveal(sess, y, "a").v
        outs.append((y.s0.v, y.s1.v, nxt.s0.v, sess.stats.as_dict(), opened))
    for i in (0, 1, 2, 4):
        _eq(outs[0][i], outs[1][i])
    st0, st1 = outs[0][3], outs[1][3]
    for k in ("rounds", "reshare_bytes", "bytes", "messages"):
        assert st0[k] == st1[k], k
    sign = [v >> (bits - 1) for v in R.to_ints(xv).tolist()]
    assert R.to_ints(outs[0][4]).tolist() == sign


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
def test_mul_trunc_many_one_launch_matches_one_by_one(bits):
    """Two independent fixed-point products in one launch (k_mul_trunc3_lat2) give bitwise
    the shares of two k_mul_trunc3_lat launches with the same seed (same nonce order)."""
    from moose_amd.runtime.session import HV

    plc = ReplicatedPlacement(owners=("a", "b", "c"))
    outs = []
    for batched in (True, False):
        sess = StackedSession("cuda", seed=5)
        if not batched:
            sess.p_mul_trunc2 = lambda *a, **k: None
        xs = [rep.share(sess, plc, HV("a", _rand(shp, bits, "cuda", i)))
              for i, shp in enumerate([(200,), (200,), (5, 40), (5, 40)])]
        r = rep.mul_trunc_many(sess, [(xs[0], xs[1], 23, None), (xs[2], xs[3], 20, None)])
        outs.append([(t.s0.v, t.s1.v) for t in r])
    for (a0, a1), (b0, b1) in zip(*outs):
        _eq(a0, b0)
        _eq(a1, b1)


@pytest.mark.gpu
def test_poly_tail_one_launch_matches_three_steps(monkeypatch):
    """A polynomial's tail (weighted sum of the powers + TruncPr + constant) in one launch
    gives bitwise the values of the three steps (seeded sigmoid: two polynomials)."""
    import moose_amd as pm

    alice, bob, carole = (pm.host_placement(n) for n in ("alice", "bob", "carole"))
    r = pm.replicated_placement("rep", players=[alice, bob, carole])

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=pm.fixed(24, 40))
        with r:
            y = pm.sigmoid(xf)
        with carole:
            return pm.cast(y, dtype=pm.float64)

    x = np.linspace(-5, 5, 61)
    got = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", seed=3,
                               use_graphs=False).evaluate_computation(f, {"x": x})
    monkeypatch.setattr(StackedSession, "p_wsum_trunc_add", lambda *a, **k: None)
    want = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", seed=3,
                                use_graphs=False).evaluate_computation(f, {"x": x})
    np.testing.assert_array_equal(list(got.values())[0], list(want.values())[0])
    np.testing.assert_allclose(list(got.values())[0], 1 / (1 + np.exp(-x)), atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("shape,nb", [((36, 200), 0), ((3, 40, 77), 1), ((5, 300), 0)])
def test_weighted_sum_device_matches_host(bits, shape, nb):
    """weighted_sum on the device (k_weighted_sum_wide for long reductions of latency-sized
    launches, k_weighted_sum otherwise) equals the host kernel."""
    k = shape[nb]
    w = [(1 << (i % 60)) + 3 * i for i in range(k)]
    a = _rand(shape, bits, "cpu", 70)
    want = R.weighted_sum(a, w, nb=nb)
    got = R.weighted_sum(R.RT(a.data.to("cuda"), bits), w, nb=nb)
    _eq(R.RT(got.data.cpu(), bits), want)


@pytest.mark.gpu
@pytest.mark.parametrize("bits,n,mirror", [(64, 301, False), (128, 300, False),
                                           (128, 37, True), (64, 4099, True)])
def test_bit_decompose_one_kernel_matches_generic(bits, n, mirror):
    """The whole of rep.bit_decompose in one kernel (StackedSession.p_bit_decompose,
    k_bitdec3) gives bitwise the shares, the nonce position and the traffic records of the
    share + slot placement + xor + AND + adder kernels (same seed, both share directions);
    the opened packed word is x itself."""
    from moose_amd.runtime.session import HV

    plc = ReplicatedPlacement(owners=("a", "b", "c"))
    outs = []
    for whole in (True, False):
        sess = StackedSession("cuda", seed=13)
        if mirror:
            sess.share_dirs = {"a": 2}
        if not whole:
            sess.p_bit_decompose = lambda *a, **k: None
        xv = _rand((n,), bits, "cuda", 9)
        x = rep.share(sess, plc, HV("b", xv))
        y = rep.bit_decompose(sess, x)
        nxt = rep.share(sess, plc, HV("b", _rand((7,), bits, "cuda", 5)))  # next nonce
        opened = rep.reveal(sess, y, "a").v
        outs.append((y.s0.v, y.s1.v, nxt.s0.v, sess.stats.as_dict(), opened, xv))
    for i in (0, 1, 2, 4):
        _eq(outs[0][i], outs[1][i])
    for k in ("rounds", "reshare_bytes", "bytes", "messages"):
        assert outs[0][3][k] == outs[1][3][k], k
    _eq(outs[0][4], outs[0][5])


@pytest.mark.gpu
@pytest.mark.parametrize("bits,n,mirror", [(64, 301, False), (128, 300, True), (128, 1001, False)])
def test_sign_arith_one_kernel_matches_generic(bits, n, mirror):
    """rep.less_than_zero_arith (b2a of the sign bit) in one kernel (StackedSession
    .p_sign_arith, k_bitdec3<SIGN>) gives bitwise the shares, nonce position and traffic
    records of the generic decomposition + bit extraction + b2a steps; it opens to [x < 0]."""
    from moose_amd.runtime.session import HV

    plc = ReplicatedPlacement(owners=("a", "b", "c"))
    outs = []
    for whole in (True, False):
        sess = StackedSession("cuda", seed=17)
        if mirror:
            sess.share_dirs = {"a": 2}
        if not whole:
            for name in ("p_sign_arith", "p_bit_decompose", "p_b2a", "p_b2a_prep"):
                setattr(sess, name, lambda *a, **k: None)
        xv = _rand((n,), bits, "cuda", 21)
        x = rep.share(sess, plc, HV("c", xv))
        y = rep.less_than_zero_arith(sess, x)
        nxt = rep.share(sess, plc, HV("b", _rand((7,), bits, "cuda", 5)))  # next nonce
        opened = rep.reveal(sess, y, "a").v
        outs.append((y.s0.v, y.s1.v, nxt.s0.v, sess.stats.as_dict(), opened, xv))
    for i in (0, 1, 2, 4):
        _eq(outs[0][i], outs[1][i])
    for k in ("rounds", "reshare_bytes", "bytes", "messages"):
        assert outs[0][3][k] == outs[1][3][k], k
    sign = [v >> (bits - 1) for v in R.to_ints(outs[0][5]).tolist()]
    assert R.to_ints(outs[0][4]).tolist() == sign


@pytest.mark.gpu
@pytest.mark.parametrize("bits,n", [(64, 301), (128, 300), (128, 70001)])
def test_mux_one_kernel_matches_generic(bits, n):
    """rep.mux(s, x, y) = s (x - y) + y in one kernel (StackedSession.p_mux, k_mux3_lat)
    gives bitwise the shares, nonce position and traffic of the sub + mul + add steps, and
    opens to the selection."""
    from moose_amd.runtime.session import HV

    plc = ReplicatedPlacement(owners=("a", "b", "c"))
    outs = []
    for whole in (True, False):
        sess = StackedSession("cuda", seed=23)
        if not whole:
            sess.p_mux = lambda *a, **k: None
        bit = R.from_ints(np.arange(n) % 2, bits, "cuda")
        s = rep.share(sess, plc, HV("a", bit))
        x = rep.share(sess, plc, HV("b", _rand((n,), bits, "cuda", 31)))
        y = rep.share(sess, plc, HV("c", _rand((n,), bits, "cuda", 32)))
        m = rep.mux(sess, s, x, y)
        nxt = rep.share(sess, plc, HV("b", _rand((7,), bits, "cuda", 5)))  # next nonce
        opened = rep.reveal(sess, m, "a").v
        outs.append((m.s0.v, m.s1.v, nxt.s0.v, sess.stats.as_dict(), opened))
    for i in (0, 1, 2, 4):
        _eq(outs[0][i], outs[1][i])
    for k in ("rounds", "reshare_bytes", "bytes", "messages"):
        assert outs[0][3][k] == outs[1][3][k], k
    xs, ys = R.to_ints(_rand((n,), bits, "cpu", 31)), R.to_ints(_rand((n,), bits, "cpu", 32))
    want = [int(xs[i]) if i % 2 else int(ys[i]) for i in range(n)]
    assert R.to_ints(outs[0][4]).tolist() == want


@pytest.mark.gpu
@pytest.mark.parametrize("bits,start,count,mirror", [(64, 0, 30, False), (128, 3, 50, True),
                                                     (128, 0, 128, False)])
def test_b2a_planes_one_kernel_matches_generic(bits, start, count, mirror):
    """rep.b2a_planes (BitSplit + b2a) in one kernel (k_b2a3 reading the packed words) gives
    bitwise the shares, nonce position and traffic records of the two steps; it opens to
    the bits of the decomposed value."""
    from moose_amd.runtime.session import HV

    plc = ReplicatedPlacement(owners=("a", "b", "c"))
    outs = []
    for whole in (True, False):
        sess = StackedSession("cuda", seed=29)
        if mirror:
            sess.share_dirs = {"a": 2}
        if not whole:
            sess.p_b2a_planes = lambda *a, **k: None
        xv = _rand((5, 41), bits, "cuda", 33)
        bd = rep.bit_decompose(sess, rep.share(sess, plc, HV("b", xv)))
        y = rep.b2a_planes(sess, bd, start, count, bits)
        nxt = rep.share(sess, plc, HV("b", _rand((7,), bits, "cuda", 5)))  # next nonce
        opened = rep.reveal(sess, y, "a").v
        outs.append((y.s0.v, y.s1.v, nxt.s0.v, sess.stats.as_dict(), opened, xv))
    for i in (0, 1, 2, 4):
        _eq(outs[0][i], outs[1][i])
    for k in ("rounds", "reshare_bytes", "bytes", "messages"):
        assert outs[0][3][k] == outs[1][3][k], k
    xs = R.to_ints(outs[0][5]).reshape(-1).tolist()
    got = R.to_ints(outs[0][4]).reshape(count, -1)
    for j in range(count):
        assert got[j].tolist() == [(v >> (start + j)) & 1 for v in xs]


@pytest.mark.gpu
@pytest.mark.parametrize("bits,n", [(64, 301), (128, 300)])
def test_negate_where_one_kernel_matches_generic(bits, n):
    """rep.negate_where(s, x) = x - 2 s x in one kernel (k_mux3_lat, absv) gives bitwise the
    shares, nonce position and traffic of mul + lincomb, and opens to -x where s = 1."""
    from moose_amd.runtime.session import HV

    plc = ReplicatedPlacement(owners=("a", "b", "c"))
    outs = []
    for whole in (True, False):
        sess = StackedSession("cuda", seed=37)
        if not whole:
            sess.p_mux = lambda *a, **k: None
        bit = R.from_ints(np.arange(n) % 2, bits, "cuda")
        s = rep.share(sess, plc, HV("a", bit))
        x = rep.share(sess, plc, HV("b", _rand((n,), bits, "cuda", 41)))
        m = rep.negate_where(sess, s, x)
        nxt = rep.share(sess, plc, HV("b", _rand((7,), bits, "cuda", 5)))  # next nonce
        opened = rep.reveal(sess, m, "a").v
        outs.append((m.s0.v, m.s1.v, nxt.s0.v, sess.stats.as_dict(), opened))
    for i in (0, 1, 2, 4):
        _eq(outs[0][i], outs[1][i])
    for k in ("rounds", "reshare_bytes", "bytes", "messages"):
        assert outs[0][3][k] == outs[1][3][k], k
    xs = R.to_ints(_rand((n,), bits, "cpu", 41))
    want = [(-int(xs[i])) % (1 << bits) if i % 2 else int(xs[i]) for i in range(n)]
    assert R.to_ints(outs[0][4]).tolist() == want


@pytest.mark.gpu
def test_exp_factors_one_launch_matches_two_steps():
    """exp's integer-part factors (MulLeading by the public vector, then + 1 on party 0's
    share) in one launch (StackedSession.p_mul_leading_add, k_mul_rows_add) give bitwise the
    shares of the two steps: whole exp(x) outputs equal with the same seed."""
    from moose_amd.protocols import fixedpoint as fxp
    from moose_amd.runtime.session import HV

    plc = ReplicatedPlacement(owners=("a", "b", "c"))
    vals = torch.linspace(-6, 3, 200, dtype=torch.float64, device="cuda")
    outs = []
    for whole in (True, False):
        sess = StackedSession("cuda", seed=43)
        if not whole:
            sess.p_mul_leading_add = lambda *a, **k: None
        x = rep.share(sess, plc, HV("a", R.encode(vals, 40, 128)))
        y = fxp.exp(sess, fxp.RepFixed(x, 40, 24))
        outs.append((y.t.s0.v, y.t.s1.v, sess.stats.as_dict()))
    _eq(outs[0][0], outs[1][0])
    _eq(outs[0][1], outs[1][1])
    assert outs[0][2]["rounds"] == outs[1][2]["rounds"]
