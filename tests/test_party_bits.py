"""Per-party fused bit decomposition front and B2A (csrc/rss_bits_party.hip, bits_party.h;
parallel/spmd.py p_bit_decompose / p_b2a_planes / p_sign_arith): with the adder over all
bits they give bitwise the shares of the generic protocol steps (share of x0 + x1, trivial
sharing of x2, xor, and, Kogge-Stone chain, sum; bit extraction, sharing, product and
linear combination of the B2A), with the same round count; with the fixed-point width
bound the sign's and exp's adders run fewer levels (fewer rounds, same result)."""
import numpy as np
import pytest

from moose_amd.protocols import fixedpoint as FP
from moose_amd.runtime.local import LocalMooseRuntime

IDS = ["alice", "bob", "carole"]


def _lr(device, monkeypatch, bits_on, width_on, one_dec=False, ring=64):
    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial

    monkeypatch.setenv("MOOSEX_PARTY_BITS", "1" if bits_on else "0")
    monkeypatch.setattr(FP, "SIGN_WIDTH", width_on)
    monkeypatch.setattr(FP, "EXP_WIDTH", width_on)
    monkeypatch.setattr(FP, "ONE_DECOMPOSITION", one_dec)
    tm = logistic_regression_tutorial(ring)
    rt = LocalMooseRuntime(IDS, device_map={i: device for i in IDS}, seed=5, use_graphs=False)
    r = np.asarray(list(rt.evaluate_computation(tm.computation, {"x": tm.x_test}).values())[0])
    return r, rt.last_stats.rounds, float(np.abs(r - tm.proba).max())


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_fused_bits_bitwise_equal_generic_steps(device, monkeypatch):
    fused, r_fused, _ = _lr(device, monkeypatch, True, False)
    generic, r_gen, _ = _lr(device, monkeypatch, False, False)
    assert np.array_equal(fused, generic)
    assert r_fused == r_gen


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_width_bound_saves_adder_levels(device, monkeypatch):
    full, r_full, e_full = _lr(device, monkeypatch, True, False)
    narrow, r_narrow, e_narrow = _lr(device, monkeypatch, True, True)
    # sign (fixed(24, 40): bit 64) and exp's integer bits (below 65): 6 levels each, not 7
    assert r_narrow == r_full - 2
    assert e_narrow < 1e-6 and e_full < 1e-6


@pytest.mark.parametrize("ring", [64, 128])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_one_decomposition_sigmoid_fused_equals_generic(device, ring, monkeypatch):
    """The sigmoid's sign and e^-|x| from one adder over x, x - T and x + T: the fused B2A
    with the sign-plane XOR and the range rows (bits_party.h plane_of) gives bitwise the
    generic Slice + BitSplit + Xor + NOT + Concat + b2a shares."""
    fused, r_fused, e = _lr(device, monkeypatch, True, True, one_dec=True, ring=ring)
    generic, r_gen, _ = _lr(device, monkeypatch, False, True, one_dec=True, ring=ring)
    assert np.array_equal(fused, generic)
    assert r_fused == r_gen and e < 1e-6


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_range_split_and_deferred_truncation_save_rounds(device, monkeypatch):
    """fixed(24, 40): the range split drops the exp tree from 32 to 8 factors (two levels
    fewer; 2 rounds, the polynomial's levels run beside the tree's); the reciprocal's last
    truncation as one dot tail whose second round merges with the reveal costs no more
    rounds than TruncPr then the mirror (and the reveal opens the truncated value only:
    tests/test_reveal_precision.py); the values stay within 1e-6 of sklearn."""
    base, r_base, e_base = _lr(device, monkeypatch, True, True, one_dec=True, ring=128)
    monkeypatch.setattr(FP, "DEFER_DOT_TRUNC", False)
    nodot, r_nodot, e_nodot = _lr(device, monkeypatch, True, True, one_dec=True, ring=128)
    monkeypatch.setattr(FP, "EXP_ONE_PRODUCT", False)
    mid, r_mid, e_mid = _lr(device, monkeypatch, True, True, one_dec=True, ring=128)
    monkeypatch.setattr(FP, "RANGE_SPLIT", False)
    monkeypatch.setattr(FP, "DEFER_OUTPUT_TRUNC", False)
    old, r_old, e_old = _lr(device, monkeypatch, True, True, one_dec=True, ring=128)
    assert r_mid == r_old - 2
    # the exp's polynomial sum and final product as one truncated product: 2 rounds fewer
    assert r_nodot == r_mid - 2
    # the dot's TruncPr left to its reader: the decomposition takes the untruncated value
    # after one reshare round instead of the tail's two
    assert r_base == r_nodot - 1
    assert max(e_base, e_nodot, e_mid, e_old) < 1e-6


def test_pending_dot_revealed_directly_and_read_by_other_ops():
    """A public-operand dot on per-party sessions keeps its TruncPr pending
    (rep.PendingTrunc): revealed directly it runs the dot tail with its second round merged
    into the reveal (2 rounds, the truncated value opened); read by another op (here a
    multiplication) it completes with the dot's tail -- both within the fixed-point error of
    the plaintext result."""
    import moose_amd as pm

    alice, bob, carole = (pm.host_placement(n) for n in IDS)
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    mir = pm.mirrored_placement(name="mir", players=[alice, bob, carole])
    fx = pm.fixed(24, 40)
    w = np.array([[0.5, -1.25], [2.0, 0.125], [-0.75, 1.0]])

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fx)
        wf = pm.cast(pm.constant(w, dtype=pm.float64, placement=mir), dtype=fx, placement=mir)
        with rep:
            y = pm.dot(xf, wf)
            z = pm.mul(pm.dot(xf, wf), pm.dot(xf, wf))
        with carole:
            return pm.cast(y, dtype=pm.float64), pm.cast(z, dtype=pm.float64)

    from moose_amd.protocols import replicated as R_

    x = np.array([[1.5, -2.0, 0.25], [3.0, 0.5, -1.0]])
    seen = []
    orig = R_._reveal_pending

    def spy(sess, v, host):
        seen.append(host)
        return orig(sess, v, host)

    R_._reveal_pending = spy
    try:
        rt = LocalMooseRuntime(IDS, device_map={i: "cpu" for i in IDS}, seed=4)
        got = [np.asarray(v) for v in rt.evaluate_computation(f, {"x": x}).values()]
    finally:
        R_._reveal_pending = orig
    p = x @ w
    for want in (p, p * p):
        assert any(g.shape == want.shape and np.abs(g - want).max() < 1e-9 for g in got)
    assert seen  # the dot revealed directly took the merged tail + reveal


def test_deferred_truncation_read_by_another_op(monkeypatch):
    """A sigmoid whose output is not revealed directly (here scaled by 2 and shifted first):
    the pending mul_add + truncation complete through the dot tail's TruncPr when the shares
    are read -- same values as the stacked simulation up to the truncation's rounding."""
    import moose_amd as pm

    alice, bob, carole = (pm.host_placement(n) for n in IDS)
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(24, 40)

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fx)
        with rep:
            s = pm.sigmoid(xf)
            y = pm.add(s, s)
        with carole:
            return pm.cast(y, dtype=pm.float64)

    x = np.array([-9.0, -2.5, -0.3, 0.0, 0.7, 3.0, 12.0, 50.0, -60.0])
    want = 2.0 / (1.0 + np.exp(-x))
    rt = LocalMooseRuntime(IDS, device_map={i: "cpu" for i in IDS}, seed=4, use_graphs=False)
    got = np.asarray(list(rt.evaluate_computation(f, {"x": x}).values())[0])
    np.testing.assert_allclose(got, want, atol=2e-6)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_one_decomposition_sigmoid_saves_rounds(device, monkeypatch):
    three, r_three, e_three = _lr(device, monkeypatch, True, True, one_dec=False)
    one, r_one, e_one = _lr(device, monkeypatch, True, True, one_dec=True)
    # sign adder and B2A (7-8) + |x| / ln 2 tail (2) + exp adder and B2A (7-8) -> one adder
    # and B2A (7-9): 10 rounds fewer for this model's fixed(14, 23)
    assert r_one <= r_three - 9
    assert e_one < 1e-6 and e_three < 1e-6
    assert np.abs(one - three).max() < 1e-6


def test_b2a_planes_xor_rows_are_abs_and_sign():
    """Generic b2a_planes_xor on a stacked session: rows = planes of |x| (x >= 0) or of
    |x| - 1 (x < 0) from the given start, then the sign plane."""
    import torch

    from moose_amd.ir.computation import ReplicatedPlacement
    from moose_amd.ops import ring as R
    from moose_amd.protocols import replicated as rep
    from moose_amd.runtime.session import HV
    from moose_amd.runtime.session import StackedSession

    sess = StackedSession("cpu", seed=3)
    plc = ReplicatedPlacement(("a", "b", "c"))
    vals = [5, -5, 0, 123456, -123456, 1]
    raw = torch.tensor([v % (1 << 64) - (1 << 64) if v % (1 << 64) >= (1 << 63) else v
                        for v in vals], dtype=torch.int64)
    x = rep.share(sess, plc, HV("a", R.RT(raw, 64)))
    bd = rep.bit_decompose(sess, x)
    ab = rep.b2a_planes_xor(sess, bd, 2, 20, 63, 64)
    got = rep.reveal(sess, ab, "c").v.data.numpy()
    assert got.shape == (21, len(vals))
    for j, v in enumerate(vals):
        a = abs(v) if v >= 0 else abs(v) - 1
        assert [int(got[r][j]) for r in range(20)] == [(a >> (r + 2)) & 1 for r in range(20)]
        assert int(got[20][j]) == (1 if v < 0 else 0)


def test_sign_bit_width_bound_is_exact_on_the_boundary(monkeypatch):
    """fixed(24, 40) values just inside |x| < 2^24 (and zero, and tiny magnitudes): the sign
    from the low 65 bits equals the true sign."""
    import moose_amd as pm

    alice, bob, carole = (pm.host_placement(n) for n in IDS)
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(24, 40)

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fx)
        with rep:
            r = pm.relu(xf)
        with carole:
            return pm.cast(r, dtype=pm.float64)

    monkeypatch.setattr(FP, "SIGN_WIDTH", True)
    x = np.array([2.0 ** 24 - 1.0, -(2.0 ** 24 - 1.0), 0.0, 2.0 ** -40, -(2.0 ** -40), 3.5, -3.5])
    rt = LocalMooseRuntime(IDS, device_map={i: "cpu" for i in IDS}, seed=2)
    got = np.asarray(list(rt.evaluate_computation(f, {"x": x}).values())[0])
    np.testing.assert_allclose(got, np.maximum(x, 0), atol=1e-9)


@pytest.mark.parametrize("ring", [64, 128])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_fused_weighted_sums_bitwise_equal_separate_steps(device, ring, monkeypatch):
    """csrc/wsum_pair: the per-party weighted sums with their public terms in one launch
    (exp's 1 - r, the polynomial sums, the sigmoid's blocks and mirror operand) give
    bitwise the shares of the separate weighted-sum / multiply / add / lincomb steps."""
    monkeypatch.setattr(FP, "WSUM_FUSED", True)
    fused, r_f, e = _lr(device, monkeypatch, True, True, one_dec=True, ring=ring)
    monkeypatch.setattr(FP, "WSUM_FUSED", False)
    sep, r_s, _ = _lr(device, monkeypatch, True, True, one_dec=True, ring=ring)
    assert np.array_equal(fused, sep) and r_f == r_s and e < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("ring", [64, 128])
def test_b2a_throughput_form_bitwise_equal_latency_form(ring, monkeypatch):
    """csrc/rss_bits_party.hip k_b2a_tp (one thread per ChaCha block, its 4 chunks'
    elements) against the latency form (a block per chunk): the same keystream chunk per
    element, so bitwise the same shares."""
    monkeypatch.delenv("MOOSEX_B2A_TP", raising=False)
    tp, r_tp, e = _lr("cuda:0", monkeypatch, True, True, one_dec=True, ring=ring)
    monkeypatch.setenv("MOOSEX_B2A_TP", "0")  # set: the latency form everywhere
    lat, r_lat, _ = _lr("cuda:0", monkeypatch, True, True, one_dec=True, ring=ring)
    assert np.array_equal(tp, lat) and r_tp == r_lat and e < 1e-6


@pytest.mark.parametrize("ring", [64, 128])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_party_mul_leading_add_bitwise_equal_steps(device, ring, monkeypatch):
    """SPMDSession.p_mul_leading_add (ring.mul_leading_add2, one mx_mul_add2 launch): exp's
    integer-part factors 1 + b_j (c_j - 1) give bitwise the shares of MulLeading on both
    components and add_public of 1 as separate steps."""
    from moose_amd.parallel.spmd import SPMDSession

    fused, r_f, e = _lr(device, monkeypatch, True, True, one_dec=True, ring=ring)
    monkeypatch.setattr(SPMDSession, "p_mul_leading_add", None)
    sep, r_s, _ = _lr(device, monkeypatch, True, True, one_dec=True, ring=ring)
    assert np.array_equal(fused, sep) and r_f == r_s and e < 1e-6


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_sigmoid_one_plus_exp_in_the_tail_equals_separate_add(device, monkeypatch):
    """The sigmoid's 1 + e^-|x|: party 0 adds 2^m * 1 to the exp's last product before its
    TruncPr (fixedpoint PLUS_IN_TAIL; a multiple of 2^m, so the truncation carries it
    exactly) -- the revealed outputs equal those of add_const after the product, bitwise,
    with no launch for the add."""
    monkeypatch.setattr(FP, "PLUS_IN_TAIL", True)
    tail, r_t, e = _lr(device, monkeypatch, True, True, one_dec=True, ring=128)
    monkeypatch.setattr(FP, "PLUS_IN_TAIL", False)
    sep, r_s, _ = _lr(device, monkeypatch, True, True, one_dec=True, ring=128)
    assert np.array_equal(tail, sep) and r_t == r_s and e < 1e-6


@pytest.mark.parametrize("ring", [64, 128])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_jobs_round2_folded_into_next_round0_bitwise_equal(device, ring, monkeypatch):
    """parallel/party.py PendingSums: a batched tail level's round-2 sums (P0's o1, P1's o0)
    written by the next level's round-0 kernel, which reads its operands through them
    (rss_jobs.hip Pend) -- bitwise the shares of the separate round-2 kernel, fewer
    launches."""
    from moose_amd.ops import ring as Rg
    from moose_amd.parallel import spmd

    calls = {"r2": 0}
    orig = Rg.jobs_r2

    def count(*a, **k):
        calls["r2"] += 1
        return orig(*a, **k)

    monkeypatch.setattr(Rg, "jobs_r2", count)
    monkeypatch.setattr(spmd, "JOBS_FOLD", True)
    fold, r_f, e = _lr(device, monkeypatch, True, True, one_dec=True, ring=ring)
    n_fold = calls["r2"]
    monkeypatch.setattr(spmd, "JOBS_FOLD", False)
    calls["r2"] = 0
    sep, r_s, _ = _lr(device, monkeypatch, True, True, one_dec=True, ring=ring)
    assert np.array_equal(fold, sep) and r_f == r_s and e < 1e-6
    assert n_fold < calls["r2"]


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_sign_beyond_the_nominal_integer_bound(device):
    """fixed(8, 27): a product keeps the nominal 8 integer bits while its value grows past
    2^8 (20 * 20 = 400).  relu / abs take the ring's msb by default (the width shortcut is
    opt-in: MOOSEX_SIGN_WIDTH=1), so the per-party runtime agrees with the stacked one and
    with the plaintext (relu(20 * 20) returned 0)."""
    import moose_amd as pm

    alice, bob, carole = (pm.host_placement(n) for n in IDS)
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(8, 27)

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fx)
        with rep:
            sq = pm.mul(xf, xf)
            r = pm.relu(pm.sub(sq, pm.constant(np.array([0.0]), dtype=fx)))
            a = pm.abs(pm.mul(xf, pm.constant(np.array([-1.0]), dtype=fx)))
        with carole:
            return pm.cast(r, dtype=pm.float64), pm.cast(a, dtype=pm.float64)

    # Z_2^128: x * x at 2^54 stays far below TruncPr's 2^126 bound (on Z_2^64 a product
    # past 2^8 would already exceed 2^62)
    x = np.array([20.0, -20.0, 21.0, 1.5, -0.25])
    outs = {}
    for name, kw in (("parties", {"device_map": {i: device for i in IDS}}),
                     ("stacked", {"device": device})):
        rt = LocalMooseRuntime(IDS, seed=2, use_graphs=False, fixedpoint_ring=128, **kw)
        outs[name] = [np.asarray(v) for v in rt.evaluate_computation(f, {"x": x}).values()]
    for name, got in outs.items():
        for want in (x * x, np.abs(x)):
            assert any(np.allclose(g, want, rtol=1e-6) for g in got), (name, got, want)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_sigmoid_beyond_the_nominal_integer_bound(device):
    """fixed(24, 40): inputs far beyond |x| < 2^24 (a product keeps the nominal integer bits
    while its value grows).  The per-party one-decomposition sigmoid takes its mirror sign
    and range flags from x itself at the ring's msb (blocks z, x - T', x + T', x), so it
    saturates to 0 / 1 like the stacked session and the plaintext (the width-
    bounded sign flipped such outputs)."""
    import moose_amd as pm

    alice, bob, carole = (pm.host_placement(n) for n in IDS)
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fx = pm.fixed(24, 40)

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fx)
        with rep:
            s = pm.sigmoid(xf)
        with bob:
            return pm.cast(s, dtype=pm.float64)

    x = np.array([3e7, -3e7, 1e10, -1e10, 5e12, -5e12, 2.5, -0.5, 0.0])
    want = 1.0 / (1.0 + np.exp(-np.clip(x, -500, 500)))
    for kw in ({"device_map": {i: device for i in IDS}}, {"device": device}):
        rt = LocalMooseRuntime(IDS, seed=3, use_graphs=False, **kw)
        got = np.asarray(list(rt.evaluate_computation(f, {"x": x}).values())[0])
        np.testing.assert_allclose(got, want, atol=1e-6, err_msg=str(kw))
