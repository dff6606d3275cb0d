"""A reveal opens exactly the declared output: the receiver's opened ring value carries the
type's fractional bits and nothing more (VERDICT r5 "what's weak" 1).

Reference: a replicated reveal sums the shares of the TruncPr'd tensor
(/root/reference/moose/src/replicated/convert.rs:280-313 after
/root/reference/moose/src/replicated/fixedpoint.rs:80-103).  The per-party sessions merge
the dot tail's second round into the reveal (parallel/party.py RoundB.reveal_to_member),
so the opened value must still be the truncated one: within TruncPr's +-1 LSB of
floor(exact / 2^m), at the type's scale."""
import numpy as np
import pytest

import moose_amd as pm
from moose_amd.ops import ring as R
from moose_amd.runtime.local import LocalMooseRuntime

IDS = ["alice", "bob", "carole"]
FX = pm.fixed(24, 40)
F = 40


def _spy_decodes(monkeypatch):
    """Record every decode: (opened ring value as signed Python ints, frac)."""
    seen = []
    orig = R.decode

    def spy(a, frac):
        if isinstance(a, R.Opened) and a.pending():
            # what the receiver holds: the sum of the addends it was sent (plus its own)
            mod = 1 << a.bits
            tot = None
            for p in a.parts:
                v = [int(t) % mod for t in R.to_ints(p).reshape(-1).tolist()]
                tot = v if tot is None else [(s + t) % mod for s, t in zip(tot, v)]
            vals = [t - mod if t >= mod // 2 else t for t in tot]
        else:
            vals = R.to_signed_ints(R.RT(a.data, a.bits)).reshape(-1).tolist()
        seen.append(([int(t) for t in vals], int(frac)))
        return orig(a, frac)

    monkeypatch.setattr(R, "decode", spy)
    return seen


def _dot_comp(host_name):
    alice, bob, carole = (pm.host_placement(n) for n in IDS)
    host = {"alice": alice, "bob": bob, "carole": carole}[host_name]
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    mir = pm.mirrored_placement(name="mir", players=[alice, bob, carole])
    w = np.array([[0.5, -1.25], [2.0, 0.125], [-0.75, 1.0]]) + 2.0 ** -30

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=FX)
        wf = pm.cast(pm.constant(w, dtype=pm.float64, placement=mir), dtype=FX, placement=mir)
        with rep:
            y = pm.dot(xf, wf)
        with host:
            return pm.cast(y, dtype=pm.float64)

    return f, w


def _enc(v):
    return [int(round(float(t) * (1 << F))) for t in np.asarray(v).reshape(-1)]


@pytest.mark.parametrize("host", IDS)
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_per_party_public_dot_reveal_has_type_precision(device, host, monkeypatch):
    """A secret x public fixed-point dot revealed directly on the per-party runtime (its
    TruncPr pending until the reveal): the opened ring value is floor(exact / 2^40) or one
    more -- not the untruncated product -- and equals the stacked session's within 1 LSB."""
    x = np.array([[1.5, -2.0, 0.25], [3.0, 0.5, -1.0]]) + 2.0 ** -33
    f, w = _dot_comp(host)
    xi = np.array(_enc(x), dtype=object).reshape(x.shape)
    wi = np.array(_enc(w), dtype=object).reshape(w.shape)
    exact = (xi.dot(wi)).reshape(-1).tolist()  # scale 2^80
    floor = [e >> F for e in exact]
    got = {}
    for name, dm in (("parties", {i: device for i in IDS}), ("stacked", None)):
        seen = _spy_decodes(monkeypatch)
        if dm is None:
            rt = LocalMooseRuntime(IDS, device=device, seed=3, use_graphs=False)
        else:
            rt = LocalMooseRuntime(IDS, device_map=dm, seed=3, use_graphs=False)
        out = np.asarray(list(rt.evaluate_computation(f, {"x": x}).values())[0])
        np.testing.assert_allclose(out, x @ w, atol=4 * 2.0 ** -F)
        reveal = [(v, fr) for v, fr in seen if len(v) == len(floor)]
        assert reveal, seen
        v, fr = reveal[-1]
        assert fr == F, f"{name}: opened with {fr} fractional bits, the type has {F}"
        assert all(0 <= a - b <= 1 for a, b in zip(v, floor)), (name, v, floor)
        got[name] = v
        monkeypatch.undo()
    assert all(abs(a - b) <= 1 for a, b in zip(got["parties"], got["stacked"]))


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_per_party_sigmoid_reveal_has_type_precision(device, monkeypatch):
    """The sigmoid's last truncation merges with the reveal (parallel/party.py MulAddTail):
    the receiver decodes at the type's 40 fractional bits, and the opened value is within a
    few LSB of the stacked session's (their polynomials differ, both ~2e-7 off sigma)."""
    alice, bob, carole = (pm.host_placement(n) for n in IDS)
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])

    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=FX)
        with rep:
            s = pm.sigmoid(xf)
        with bob:
            return pm.cast(s, dtype=pm.float64)

    x = np.array([-9.0, -2.5, -0.3, 0.0, 0.7, 3.0, 12.0])
    want = 1.0 / (1.0 + np.exp(-x))
    vals = {}
    for name in ("parties", "stacked"):
        seen = _spy_decodes(monkeypatch)
        if name == "stacked":
            rt = LocalMooseRuntime(IDS, device=device, seed=3, use_graphs=False)
        else:
            rt = LocalMooseRuntime(IDS, device_map={i: device for i in IDS}, seed=3,
                                   use_graphs=False)
        out = np.asarray(list(rt.evaluate_computation(f, {"x": x}).values())[0])
        np.testing.assert_allclose(out, want, atol=1e-6)
        reveal = [(v, fr) for v, fr in seen if len(v) == len(x)]
        v, fr = reveal[-1]
        assert fr == F, f"{name}: opened with {fr} fractional bits, the type has {F}"
        assert all(abs(a) <= (1 << F) + 4 for a in v)  # a probability at 2^40
        vals[name] = v
        monkeypatch.undo()
    assert max(abs(a - b) for a, b in zip(vals["parties"], vals["stacked"])) < 2e-6 * (1 << F)
