"""The per-party fixed-point dot tail (parallel/party.py, csrc/rss_party.hip): the dot's
reshare folded into TruncPr's first round gives bitwise the same shares as the protocol
steps it replaces (zero share + reshare + TruncPr; reference replicated/arith.rs:436-492,
replicated/fixedpoint.rs:80-103) with 2 rounds instead of 3."""
import pytest
import torch

from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ops import ring as R
from moose_amd.protocols import replicated as rep
from moose_amd.runtime.session import HV
from moose_amd.runtime.session import StackedSession

PLC = ReplicatedPlacement(("a", "b", "c"))


def _operands(bits, m=40, k=24, n=16, device="cpu"):
    g = torch.Generator().manual_seed(bits)
    a = torch.rand(m, k, generator=g, dtype=torch.float64) * 6 - 3
    b = torch.rand(k, n, generator=g, dtype=torch.float64) * 4 - 2
    enc = lambda t: R.RT(R.to_device(R.encode(t, 23, bits).data, device), bits)  # noqa: E731
    return a, b, HV("a", enc(a)), HV("b", enc(b))


def _run(monkeypatch, bits, tail, chunks=1, device="cpu", fused=False):
    monkeypatch.setenv("MOOSEX_DOT_TAIL", "1" if tail else "0")
    s = StackedSession(device, seed=3)
    s.fused = fused
    s.pipeline_chunks = chunks
    a, b, xa, yb = _operands(bits, m=128 * chunks + 40, device=device)
    X, Y = rep.share(s, PLC, xa), rep.share(s, PLC, yb)
    r0 = s.stats.rounds
    Z = rep.dot_trunc(s, X, Y, 23)
    rounds = s.stats.rounds - r0
    out = R.decode(R.RT(rep.reveal(s, Z, "c").v.data.cpu(), bits), 23)
    return Z, rounds, out, a @ b


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("chunks", [1, 4])
def test_party_tail_bitwise_equals_reshare_then_truncpr(monkeypatch, bits, chunks):
    new, r_new, out, want = _run(monkeypatch, bits, True, chunks)
    old, _, _, _ = _run(monkeypatch, bits, False, chunks)
    assert torch.equal(new.s0.v.data, old.s0.v.data)
    assert torch.equal(new.s1.v.data, old.s1.v.data)
    assert r_new == 2 * chunks  # per chunk: round A (reshare folded in) + round B
    assert (out - want).abs().max() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
def test_party_tail_gpu_matches_fused_and_cpu(monkeypatch, bits):
    """Device per-party kernels (all three roles in one launch) == the stacked fused
    single-kernel tail == the host per-party kernels."""
    cpu, _, _, _ = _run(monkeypatch, bits, True)
    fused, _, _, _ = _run(monkeypatch, bits, True, device="cuda", fused=True)
    party, _, _, _ = _run(monkeypatch, bits, True, device="cuda", fused=False)
    for t in (fused, party):
        assert torch.equal(t.s0.v.data.cpu(), cpu.s0.v.data)
        assert torch.equal(t.s1.v.data.cpu(), cpu.s1.v.data)
