"""Key slots (runtime/keys.py, csrc/moosex.h): PRF evaluations with keys read from a
device key table are bit-identical to the same PRFs with host-expanded keys, and a
refreshed table yields different randomness."""
import os

import pytest
import torch

from moose_amd.ops import ring as R
from moose_amd.runtime.keys import KeyTable



def _table(device, keys):
    kt = KeyTable(device, capacity=8)
    kt._write(0, keys)
    kt.n = len(keys)
    return kt


def _devices():
    return [pytest.param("cpu")] + [pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("device", _devices())
@pytest.mark.parametrize("bits", [1, 64, 128])
def test_rss_cross_slots_match_host_keys(device, bits):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    keys = [os.urandom(16) for _ in range(3)]
    kt = _table(device, keys)
    shape = (3, 37, 5)
    x0, x1, y0, y1 = (R.prf_expand([os.urandom(16)], 1, shape, bits, device) for _ in range(4))
    x0, x1, y0, y1 = (R.RT(t.data[0], bits) for t in (x0, x1, y0, y1))
    kind = "bool" if bits == 1 else "arith"
    ref = R.rss_cross(kind, x0, x1, y0, y1, keys + [keys[0]], 7, 3)
    got = R.rss_cross_k(kind, x0, x1, y0, y1, kt.ptr(0), 3, 7, 3)
    assert torch.equal(ref.data.cpu(), got.data.cpu())
    zs = R.rss_cross_k(kind, R.zeros(shape, bits, device), None, None, None, kt.ptr(0), 3, 9, 3)
    ref_zs = R.rss_cross(kind, R.zeros(shape, bits, device), None, None, None,
                         keys + [keys[0]], 9, 3)
    assert torch.equal(zs.data.cpu(), ref_zs.data.cpu())


@pytest.mark.parametrize("device", _devices())
@pytest.mark.parametrize("bits", [1, 64, 128])
def test_prf_expand_slots_match_host_keys(device, bits):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    keys = [os.urandom(16) for _ in range(2)]
    kt = _table(device, keys)
    ref = R.prf_expand(keys, 5, (10, 3), bits, device)
    got = R.prf_expand_k(kt.ptr(0), 2, 5, (10, 3), bits, device)
    assert torch.equal(ref.data.cpu(), got.data.cpu())
    one = R.prf_expand_k(kt.ptr(1), 1, 5, (10, 3), bits, device)
    assert torch.equal(one.data[0].cpu(), ref.data[1].cpu())


def test_refresh_changes_keys_and_randomness():
    kt = KeyTable("cpu", capacity=4)
    base = kt.alloc(2)
    before = kt.raw_key(base)
    a = R.prf_expand_k(kt.ptr(base), 1, 1, (64,), 64, "cpu")
    kt.refresh()
    assert kt.raw_key(base) != before
    b = R.prf_expand_k(kt.ptr(base), 1, 1, (64,), 64, "cpu")
    assert not torch.equal(a.data, b.data)


def test_frozen_table_does_not_write():
    kt = KeyTable("cpu", capacity=4)
    kt.refresh()
    snap = kt.t.clone()
    kt.frozen = True
    kt.alloc(3)
    assert torch.equal(snap, kt.t)
    with pytest.raises(RuntimeError):
        kt.alloc(2)


@pytest.mark.parametrize("device", _devices())
@pytest.mark.parametrize("bits", [1, 64, 128])
def test_fused_mul_reshare_matches_cross_then_shift(device, bits):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    keys = [os.urandom(16) for _ in range(3)]
    kt = _table(device, keys)
    shape = (3, 9, 4)
    x0, x1, y0, y1 = (R.RT(R.prf_expand([os.urandom(16)], 1, shape, bits, device).data[0], bits)
                      for _ in range(4))
    kind = "bool" if bits == 1 else "arith"
    z = R.rss_cross_k(kind, x0, x1, y0, y1, kt.ptr(0), 3, 11, 3)
    s0, s1 = R.rss_mul3_k(kind, x0, x1, y0, y1, kt.ptr(0), 11)
    assert torch.equal(s0.data.cpu(), z.data.cpu())
    assert torch.equal(s1.data.cpu(), torch.roll(z.data, -1, dims=0).cpu())


@pytest.mark.gpu
def test_device_key_refresh_matches_host_derivation():
    """KeyTable.refresh_device (csrc/party_graph.hip): slot s of the e-th refresh holds the
    first 16 bytes of ChaCha12(master, nonce e, block s) and that key's AES-128 schedule --
    the host derivation (mx_key_refresh_host) and the host slot image (mx_key_slots) of the
    same key -- and every refresh gives new keys."""
    import ctypes

    import numpy as np

    from moose_amd.ops import native as nat
    from moose_amd.runtime.keys import slot_words

    kt = KeyTable("cuda:0", capacity=40)
    kt.enable_device_refresh()
    master = kt._master.cpu().numpy().view(np.uint32).copy()
    seen = set()
    for e in range(3):
        kt.refresh_device(37)
        got = kt.t.cpu().numpy().view(np.uint32)
        assert int(kt._epoch.item()) == e + 1
        for s in (0, 1, 17, 36):
            want = np.zeros(48, dtype=np.uint32)
            nat.lib().mx_key_refresh_host(master.ctypes.data_as(ctypes.c_void_p), e, s,
                                          want.ctypes.data_as(ctypes.c_void_p))
            assert np.array_equal(got[s], want), (e, s)
            raw = got[s, :4].tobytes()
            assert np.array_equal(slot_words([raw])[0], want)  # the host AES schedule
            seen.add(raw)
        assert not got[37:].any()  # slots past the refreshed range untouched
    assert len(seen) == 12
    torch.cuda.synchronize()
