"""Cyclic multi-GPU layout (moose_amd/parallel/cyclic.py) over gloo: N ranks, N sessions,
each party of a session on a different rank.  Every component of every rank must be
bitwise equal to the same party of a single-process stacked session run with that
session's keys -- i.e. moving the parties apart changed where the data lives, not what it
is.  (Reference strategy: the per-worker integration runs of ``moose/src/execution``
compared against the in-process runtime.)"""
import os
import queue
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from moose_amd.ir.computation import ReplicatedPlacement
from moose_amd.ops import ring as R

PLC = ReplicatedPlacement(("a", "b", "c"))
SEED = 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(session, bits):
    v = torch.linspace(-20, 20, 96, dtype=torch.float64) + 0.25 * session
    return R.encode(v, 23, bits)


def _mats(session, bits, big=False):
    """(256 x 16) . (16 x 8) operands for the row-chunked dot+TruncPr pipeline; ``big``:
    (256 x 256) . (256 x 256), large enough for the asymmetric local products."""
    k, n = (256, 256) if big else (16, 8)
    a = torch.linspace(-3, 3, 256 * k, dtype=torch.float64).reshape(256, k) + 0.1 * session
    b = torch.linspace(-2, 2, k * n, dtype=torch.float64).reshape(k, n) - 0.05 * session
    return R.encode(a / (k / 16), 23, bits), R.encode(b, 23, bits)


def _program(sess, xb, ya, mb, ma):
    """share (owners b and a), mul + trunc, dot, bit decomposition, reveal to c; a
    pipelined fixed-point matrix product (2 row chunks) revealed to c."""
    from moose_amd.protocols import replicated as rep

    X = rep.share(sess, PLC, xb)
    Y = rep.share(sess, PLC, ya)
    M = rep.trunc_pr(sess, rep.mul(sess, X, Y), 23)
    D = rep.dot(sess, rep.local(sess, X, "Reshape", shape=(8, 12)),
                rep.local(sess, Y, "Reshape", shape=(12, 8)))
    B = rep.bit_decompose(sess, X)
    DT = rep.dot_trunc(sess, rep.share(sess, PLC, mb), rep.share(sess, PLC, ma), 23)
    out = rep.reveal(sess, M, "c")
    dt = rep.reveal(sess, DT, "c")
    tensors = [t.s0.v.data.clone() for t in (X, Y, M, D, B, DT)] + [
        t.s1.v.data.clone() for t in (X, Y, M, D, B, DT)]
    return tensors, (out.v.data.clone(), dt.v.data.clone())


def _worker(rank, world, port, q, device="cpu", offsets=None, chunks=4, dirs=None,
            backend="gloo", big=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":  # one GPU per rank, every exchange an RCCL send/recv
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(rank)
        device = f"cuda:{rank}"
    dist.init_process_group(backend, rank=rank, world_size=world)
    from moose_amd.parallel.cyclic import CyclicSession
    from moose_amd.parallel.cyclic import RingComm
    from moose_amd.runtime.session import HV

    sess = CyclicSession(RingComm(rank, world, device), offsets or {"a": 0, "b": 1, "c": 2},
                         seed=SEED,
                         device=device, pipeline_chunks=chunks, share_dirs=dirs)
    res = {}
    for bits in (64, 128):
        xd, yd = _data(sess.session_of("b"), bits), _data(100 + sess.session_of("a"), bits)
        xb = HV("b", R.RT(R.to_device(xd.data, device), bits))
        ya = HV("a", R.RT(R.to_device(yd.data, device), bits))
        ma_, _ = _mats(sess.session_of("b"), bits, big)
        _, mb_ = _mats(sess.session_of("a"), bits, big)
        mb = HV("b", R.RT(R.to_device(ma_.data, device), bits))
        ma = HV("a", R.RT(R.to_device(mb_.data, device), bits))
        ts, outs = _program(sess, xb, ya, mb, ma)
        res[bits] = ([t.cpu().numpy() for t in ts], [o.cpu().numpy() for o in outs],
                     sess.session_of("c"))
    keys = {s: sess.session_keys(PLC, s) for s in range(world)}
    q.put((rank, res, keys, sess.comm.messages))
    dist.barrier()
    dist.destroy_process_group()


def _stacked_reference(keys, session, chunks=4, dirs=None, big=False):
    """The worker's program for both ring widths, in the same order (one nonce stream)."""
    from moose_amd.runtime.session import HV
    from moose_amd.runtime.session import StackedSession

    s = StackedSession("cpu", seed=1)
    s.fused = False
    s.pipeline_chunks = chunks
    if dirs:
        s.share_dirs = dirs
    base = s.setup(PLC)
    s.keytable._write(base, keys)
    out = {}
    for bits in (64, 128):
        xb = HV("b", _data(session, bits))
        ya = HV("a", _data(100 + session, bits))
        ma_, mb_ = _mats(session, bits, big)
        out[bits] = _program(s, xb, ya, HV("b", ma_), HV("a", mb_))
    return out


def _run(world, device, offsets=None, chunks=4, dirs=None, backend="gloo", big=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, device, offsets, chunks, dirs,
                                            backend, big)) for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    deadline = time.monotonic() + 300
    while len(got) < world:  # fail fast if a worker died instead of waiting out a timeout
        try:
            rank, res, keys, msgs = q.get(timeout=2)
            got[rank] = (res, keys, msgs)
        except queue.Empty:
            dead = [p.exitcode for p in ps if p.exitcode not in (None, 0)]
            if dead or time.monotonic() > deadline:
                for p in ps:
                    p.kill()
                raise AssertionError(f"cyclic workers failed: exit codes {dead}")
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    keys = got[0][1]
    refs = {}
    for s in range(world):
        r = _stacked_reference(keys[s], s, chunks, dirs, big)
        refs.update({(s, b): r[b] for b in (64, 128)})
    for g in range(world):
        res, _, msgs = got[g]
        assert msgs > 0  # the parties really exchanged messages
        for bits in (64, 128):
            ts, out, s_c = res[bits]
            for i, t in enumerate(ts):
                for p in range(3):
                    # component p of rank g = party p of session g - o(p)
                    s = (g - (offsets or {}).get("abc"[p], p)) % world
                    ref = refs[(s, bits)][0][i][p].numpy()
                    assert np.array_equal(t[p], ref), (world, g, bits, i, p)
            # carole's revealed products on rank g are session g - o(c)'s
            for o, r in zip(out, refs[(s_c, bits)][1]):
                assert np.array_equal(o, r.numpy())
            x = _data(s_c, bits)
            y = _data(100 + s_c, bits)
            want = R.decode(x, 23) * R.decode(y, 23)
            np.testing.assert_allclose(
                R.decode(R.RT(torch.from_numpy(out[0]), bits), 23).numpy(), want.numpy(),
                atol=1e-5)
            ma_, mb_ = _mats(s_c, bits, big)
            want = R.decode(ma_, 23).numpy() @ R.decode(mb_, 23).numpy()
            np.testing.assert_allclose(
                R.decode(R.RT(torch.from_numpy(out[1]), bits), 23).numpy(), want, atol=1e-4)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_cyclic_bitwise_equals_stacked(world):
    _run(world, "cpu")


def test_cyclic_asym_products_bitwise_equals_stacked():
    """Three ranks, a 256^3 product unchunked: every component takes the asymmetric local
    products of its party (two-stack form) and the shares still equal the stacked
    session's bit for bit."""
    _run(3, "cpu", chunks=1, big=True)


def test_cyclic_unchunked_dealer_early():
    """Unchunked dot_trunc: the dealer's rt1 / rm1 go out before the GEMM
    (party.dealer_early) -- still bitwise the stacked session's shares."""
    _run(3, "cpu", chunks=1)


def test_cyclic_mirrored_share_direction():
    """Input sharing towards P_{j+2} (share_dir 2, as default_layout picks on 8 GPUs) for
    owner b, unchunked tail: bitwise the stacked session's shares under the same choice."""
    _run(4, "cpu", {"a": 0, "b": 1, "c": 3}, chunks=1, dirs={"b": 2})


def test_cyclic_link_balanced_offsets():
    """The link-balanced placement bench.py uses on >= 4 GPUs: on 8 GPUs carole at offset
    3, so every inter-party flow of the dot program has its own xGMI link (busiest link 2.5
    share tensors per step instead of 4.5 with offsets 0, 1, 2)."""
    from moose_amd.parallel.cyclic import default_layout
    from moose_amd.parallel.cyclic import link_loads

    off8, dirs8 = default_layout(("a", "b", "c"), 8)
    assert off8 == {"a": 0, "b": 1, "c": 3} and dirs8 == {}
    assert max(link_loads((0, 1, 3), 8).values()) == 2.5 < max(link_loads((0, 1, 2), 8).values())
    off4, dirs4 = default_layout(("a", "b", "c"), 4)
    assert max(link_loads(list(off4.values()), 4).values()) == 3.5
    assert default_layout(("a", "b", "c"), 2) == ({"a": 0, "b": 1, "c": 2}, {})
    _run(4, "cpu", off4, dirs=dirs4)


@pytest.mark.gpu
def test_cyclic_on_gpu_bitwise_equals_cpu_stacked():
    """Three party processes sharing the one test GPU (payloads staged through gloo):
    the per-party key-pair kernels and the layout's data movement run on the device and
    must reproduce the CPU stacked reference bit for bit."""
    _run(3, "cuda:0")


@pytest.mark.gpu
@pytest.mark.skipif(torch.cuda.device_count() < 3, reason="RCCL across GPUs: needs >= 3 GPUs")
@pytest.mark.parametrize("world", [3, 4])
def test_cyclic_rccl_multi_gpu_bitwise_equals_cpu_stacked(world):
    """One rank per GPU over RCCL (backend "nccl"): every reshare, dealer message and
    reveal crosses xGMI, and the shares are bit for bit the CPU stacked session's
    (multi-GPU RCCL tests gated on the device count)."""
    if torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs")
    _run(world, "cuda", backend="nccl")
