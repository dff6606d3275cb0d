"""The reveal's lazy sum (ops/ring.py ``Opened``): decoding a revealed value runs one fused
add + decode pass (mx_addn_decode) and must equal add3 followed by decode; any other use
materialises the ring-valued sum (reference reveal: replicated/convert.rs:280-313, decode:
host/fixedpoint.rs)."""
import pytest
import torch

from moose_amd.ops import ring as R


def _parts(bits, device):
    g = torch.Generator().manual_seed(bits)
    x = torch.rand(33, 17, generator=g, dtype=torch.float64) * 10 - 5
    e = R.encode(x, 23, bits)
    a = R.RT(torch.randint(-2**62, 2**62, e.data.shape, dtype=torch.int64, generator=g), bits)
    b = R.RT(torch.randint(-2**62, 2**62, e.data.shape, dtype=torch.int64, generator=g), bits)
    c = R.binary("sub", R.binary("sub", e, a), b)
    mv = lambda t: R.RT(t.data.to(device), bits)  # noqa: E731
    return x, mv(a), mv(b), mv(c)


def _check(bits, device):
    x, a, b, c = _parts(bits, device)
    o = R.opened(a, b, c)
    assert isinstance(o, R.Opened) and o.shape == a.shape and o.pending()
    fused = R.decode(o, 23)
    assert o.pending()  # the fused decode did not form the sum
    want = R.decode(R.add3(a, b, c), 23)
    assert torch.equal(fused, want)
    assert (fused.cpu() - x).abs().max() < 1e-6
    assert torch.equal(o.data, R.add3(a, b, c).data) and not o.pending()
    assert torch.equal(R.decode(o, 23), want)


@pytest.mark.parametrize("bits", [64, 128])
def test_opened_decode_equals_add3_then_decode(bits):
    _check(bits, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [64, 128])
def test_opened_decode_gpu(bits):
    _check(bits, "cuda")


@pytest.mark.gpu
def test_lazy_values_cross_streams():
    """A lazy value made on one stream and consumed on another: the consumer orders itself
    after the producer stream (ring._join), for Opened (fused decode) and Encoded (fused
    share source and materialisation)."""
    x, a, b, c = _parts(128, "cuda")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        big = torch.full((1 << 24,), 3.0, device="cuda")
        for _ in range(20):  # keep the side stream busy before the parts are written
            big = big * 1.0000001
        c2 = R.RT(c.data.clone(), 128)
        o = R.opened(a, b, c2)
        e = R.encode_lazy(x.cuda(), 23, 128)
    got = R.decode(o, 23)  # on the default stream
    assert (got.cpu() - x).abs().max() < 1e-6
    assert torch.equal(e.data.cpu(), R.encode(x, 23, 128).data)
