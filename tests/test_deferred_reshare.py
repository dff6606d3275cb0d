"""The cyclic layout's deferred last reshare (protocols/replicated.py DeferredRep,
parallel/party.py RoundB): a product consumed by another product completes its shares
first; a product revealed to the dealer P2 merges the round into the reveal.  Both must
give bitwise the stacked session's shares and outputs (one process: the cyclic session on
one rank, same keys)."""
import pytest
import torch

from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ops import ring as R
from moose_amd.protocols import replicated as rep
from moose_amd.runtime.session import HV
from moose_amd.runtime.session import StackedSession

PLC = ReplicatedPlacement(("a", "b", "c"))


def _program(sess, bits):
    g = torch.Generator().manual_seed(bits)
    mats = [torch.rand(s, generator=g, dtype=torch.float64) * 2 - 1
            for s in ((32, 16), (16, 16), (16, 8))]
    enc = lambda t: R.encode(t, 23, bits)  # noqa: E731
    X = rep.share(sess, PLC, HV("a", enc(mats[0])))
    Y = rep.share(sess, PLC, HV("b", enc(mats[1])))
    V = rep.share(sess, PLC, HV("a", enc(mats[2])))
    Z = rep.dot_trunc(sess, X, Y, 23)        # consumed by a product: completed first
    W = rep.dot_trunc(sess, Z, V, 23)        # revealed to the dealer: merged round
    out_w = rep.reveal(sess, W, "c").v
    out_z = rep.reveal(sess, Z, "a").v       # a reveal to another party: completed
    dec = lambda v: R.decode(R.RT(v.data, bits), 23)  # noqa: E731
    merged = isinstance(W, rep.DeferredRep) and W._tail.done is False
    return ([Z.s0.v.data.clone(), Z.s1.v.data.clone(), W.s0.v.data.clone(),
             W.s1.v.data.clone()], dec(out_w), dec(out_z), mats, merged)


@pytest.mark.parametrize("bits", [64, 128])
def test_deferred_reshare_bitwise(bits):
    from moose_amd.parallel.cyclic import CyclicSession
    from moose_amd.parallel.cyclic import RingComm

    cyc = CyclicSession(RingComm(0, 1, "cpu"), {"a": 0, "b": 1, "c": 2}, "cpu", seed=9,
                        pipeline_chunks=1)
    assert cyc.defer_reshare
    keys = cyc.session_keys(PLC, 0)
    st = StackedSession("cpu", seed=9)
    st.fused = False
    st.keytable._write(st.setup(PLC), keys)
    got, wc, zc, mats, merged = _program(cyc, bits)
    ref, wr, zr, _, _ = _program(st, bits)
    assert merged  # W's reveal to c took the merged round (its shares were completed later)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    assert torch.equal(wc, wr) and torch.equal(zc, zr)
    want = mats[0] @ mats[1] @ mats[2]
    assert (wc - want).abs().max() < 1e-4
