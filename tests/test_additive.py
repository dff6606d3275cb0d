"""Additive (2-party) dialect: sharing, linear ops, rep<->adt conversions, dealer DaBits
and probabilistic truncation (reference ``additive/*`` unit tests)."""
import numpy as np
import pytest
import torch

from moose_amd.ir.computation import AdditivePlacement
from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ops import ring as R
from moose_amd.protocols import additive as adt
from moose_amd.protocols import replicated as rep
from moose_amd.runtime.session import HV
from moose_amd.runtime.session import StackedSession

RP = ReplicatedPlacement(("a", "b", "c"))
AP = AdditivePlacement(("a", "b"))


@pytest.fixture(params=[64, 128])
def bits(request):
    return request.param


def _ints(xs, bits):
    return R.from_ints([v % (1 << bits) for v in xs], bits)


def test_share_reveal_linear(bits):
    s = StackedSession("cpu", seed=1)
    xs, ys = [5, -7, 1 << 40, 0], [1, 2, 3, -4]
    for owner in ("a", "b", "c"):
        X = adt.share(s, AP, HV(owner, _ints(xs, bits)))
        Y = adt.share(s, AP, HV("b", _ints(ys, bits)))
        got = R.to_signed_ints(adt.reveal(s, adt.add(s, X, Y), "c").v)
        assert list(got) == [x + y for x, y in zip(xs, ys)]
        got = R.to_signed_ints(adt.reveal(s, adt.sub(s, X, adt.neg(s, Y)), "a").v)
        assert list(got) == [x + y for x, y in zip(xs, ys)]
        got = R.to_signed_ints(adt.reveal(s, adt.shl(s, adt.mul_public(s, X, _ints([3], bits)), 1),
                                          "a").v)
        assert list(got) == [6 * x for x in xs]


def test_rep_adt_rep_roundtrip(bits):
    s = StackedSession("cpu", seed=2)
    xs = [11, -3, 1 << 33, 7]
    X = rep.share(s, RP, HV("c", _ints(xs, bits)))
    A = adt.from_rep(s, X)
    assert list(R.to_signed_ints(adt.reveal(s, A, "c").v)) == xs
    back = adt.to_rep(s, RP, A)
    assert list(R.to_signed_ints(rep.reveal(s, back, "a").v)) == xs
    # a different owner pair of the replicated placement
    A2 = adt.from_rep(s, X, AdditivePlacement(("c", "a")))
    assert list(R.to_signed_ints(adt.reveal(s, A2, "b").v)) == xs


def test_trunc_pr_error_bound(bits):
    s = StackedSession("cpu", seed=3)
    xs = np.arange(-5000, 5000, 7) * 1009
    A = adt.from_rep(s, rep.share(s, RP, HV("a", _ints(xs.tolist(), bits))))
    T = adt.trunc_pr(s, RP, A, 12, [s.nonce(RP) for _ in range(4)])
    got = R.to_signed_ints(adt.reveal(s, T, "a").v).astype(np.float64)
    assert np.abs(got - np.floor(xs / 4096)).max() <= 1


def test_dabit(bits):
    s = StackedSession("cpu", seed=4)
    shape = HV("a", (1000,))
    A, B = adt.dabit(s, RP, shape, bits, [s.nonce(RP) for _ in range(3)])
    a = R.to_ints(adt.reveal(s, A, "c").v)
    b = adt.reveal(s, B, "c").v.data.numpy()
    assert set(np.unique(b).tolist()) <= {0, 1} and 300 < b.sum() < 700
    np.testing.assert_array_equal(np.asarray(a, dtype=np.int64), b.astype(np.int64))


def test_rep_trunc_uses_additive_and_matches_fused(bits):
    outs = []
    for fused in (False, True):
        s = StackedSession("cpu", seed=5)
        s.fused = fused
        X = rep.share(s, RP, HV("b", R.encode(torch.linspace(-9, 9, 77, dtype=torch.float64), 23,
                                              bits)))
        T = rep.trunc_pr(s, rep.mul(s, X, X), 23)
        outs.append((T.s0.v.data.clone(), T.s1.v.data.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
