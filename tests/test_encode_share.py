"""Input sharing of a deferred fixed-point encoding (ops/ring.py ``Encoded``): the share
kernels encode the float64 input themselves (kind MX_SHARE_F64) and must produce bitwise
the shares of encode-then-share, in the stacked fused kernel and in the per-party kernel
(reference: host/fixedpoint.rs encode + replicated/convert.rs:74-90 share)."""
import pytest
import torch

from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ops import ring as R
from moose_amd.protocols import replicated as rep
from moose_amd.runtime.session import HV
from moose_amd.runtime.session import StackedSession

PLC = ReplicatedPlacement(("a", "b", "c"))


def _x(device):
    g = torch.Generator().manual_seed(7)
    return (torch.rand(37, 11, generator=g, dtype=torch.float64) * 200 - 100).to(device)


def _shares(bits, device, lazy, fused, owner, dirs=None, keys=None):
    if fused == "generic":  # the protocol-level path (host PRF + sub + move)
        s = StackedSession(device, seed=11)
        s.fused = False
    elif fused:  # stacked session: the whole-sharing kernel (mx_share3_k)
        s = StackedSession(device, seed=11)
    else:  # the per-party kernel (mx_share_party), the cyclic layout on one device
        from moose_amd.parallel.cyclic import CyclicSession
        from moose_amd.parallel.cyclic import RingComm

        s = CyclicSession(RingComm(0, 1, device), {"a": 0, "b": 1, "c": 2}, device, seed=11)
    if keys is not None:  # a stacked session on the cyclic session's keys (k0, k1, k2, k_all)
        s.keytable._write(s.setup(PLC), keys)
    if dirs:
        s.share_dirs = dirs
    x = _x(device)
    v = R.encode_lazy(x, 23, bits) if lazy else R.encode(x, 23, bits)
    assert isinstance(v, R.Encoded) == (lazy and bits in (64, 128))
    X = rep.share(s, PLC, HV(owner, v))
    if lazy:
        assert v.pending()  # the kernel encoded the input; the encoding was never formed
    out = R.decode(R.RT(rep.reveal(s, X, "c").v.data, bits), 23)
    return X.s0.v.data, X.s1.v.data, out, x


def _check(bits, device, fused, owner):
    a0, a1, out, x = _shares(bits, device, True, fused, owner)
    b0, b1, _, _ = _shares(bits, device, False, fused, owner)
    assert torch.equal(a0, b0) and torch.equal(a1, b1)
    assert (out.cpu() - x.cpu()).abs().max() < 1e-6


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("owner", ["a", "c"])
def test_encode_in_share_kernel_bitwise(bits, fused, owner):
    _check(bits, "cpu", fused, owner)


@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("owner", ["a", "b"])
def test_mirrored_share_direction_all_paths_agree(bits, owner):
    """share_dir 2 (the masked slot to P_{j+2}): the stacked kernel, the per-party kernel
    and the protocol-level path give the same shares, and differ from direction 1."""
    from moose_amd.parallel.cyclic import CyclicSession
    from moose_amd.parallel.cyclic import RingComm

    dirs = {owner: 2}
    keys = CyclicSession(RingComm(0, 1, "cpu"), {"a": 0, "b": 1, "c": 2}, "cpu",
                         seed=11).session_keys(PLC, 0)
    got = [_shares(bits, "cpu", lazy, f, owner, dirs, None if f is False else keys)
           for f, lazy in (("generic", False), (True, True), (False, True))]
    for a0, a1, out, x in got[1:]:
        assert torch.equal(a0, got[0][0]) and torch.equal(a1, got[0][1])
        assert (out - x).abs().max() < 1e-6
    ref = _shares(bits, "cpu", True, True, owner)
    assert not torch.equal(ref[0], got[0][0])


def test_encoded_materialises_on_use():
    x = _x("cpu")
    v = R.encode_lazy(x, 23, 128)
    assert torch.equal(v.data, R.encode(x, 23, 128).data) and not v.pending()


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
@pytest.mark.parametrize("fused", [True, False])
def test_encode_in_share_kernel_gpu(bits, fused):
    _check(bits, "cuda", fused, "b")
