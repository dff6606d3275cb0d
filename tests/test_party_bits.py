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


def _lr(device, monkeypatch, bits_on, width_on):
    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial

    monkeypatch.setenv("MOOSEX_PARTY_BITS", "1" if bits_on else "0")
    monkeypatch.setattr(FP, "SIGN_WIDTH", width_on)
    tm = logistic_regression_tutorial(16)
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
