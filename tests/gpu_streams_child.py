"""Per-party stream-graph checks that need the party streams on distinct hardware queues.

A HIP stream is served by one of the process's hardware queues (GPU_MAX_HW_QUEUES, 4 by
default).  A flag wait (csrc/party_graph.hip k_wait) spins on the device until its producer
writes the flag; if the producer's kernels sit on the SAME queue behind the wait, the wait
can only time out.  In a long test process the streams' queue assignment depends on every
stream created before, so tests/test_threads.py runs these checks in a fresh child process
(this file, ``python tests/gpu_streams_child.py <case>``) with more hardware queues than the
process has streams: every party stream then has a queue to itself, and the checks FAIL
(exit 1) instead of skipping when the wait times out.

Cases:
  flag      k_push / k_wait ordering of two graphs on two streams (5 replays)
  replay    seeded per-party stream graphs: capture-time validation passes, every replay
            bitwise equal to eager, no fallback
  fault     a corrupted landing buffer (MOOSEX_FAULT=party_landing) is caught by the
            validation (wrong values, not a timeout) and the per-action replay is kept
  fallback  a lost message after the validation: the per-action replay from then on
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def flag_case():
    from moose_amd.ops import native as nat

    dev = torch.device("cuda:0")
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    n = 4096
    val = torch.zeros(1, dtype=torch.int64, device=dev)
    payload = torch.zeros(n, dtype=torch.int64, device=dev)
    landing = nat.uncached_zeros((n,), torch.int64, dev)
    out = torch.zeros(n, dtype=torch.int64, device=dev)
    m = torch.randn(1 << 24, device=dev)
    torch.sin(m)
    ga, gb = torch.cuda.CUDAGraph(keep_graph=True), torch.cuda.CUDAGraph(keep_graph=True)
    torch.cuda.synchronize()
    with torch.cuda.stream(sa):
        ga.capture_begin()
        y = m
        for _ in range(40):  # ~1 ms of work before the payload is written
            y = torch.sin(y)
        payload.copy_(val.expand(n) + (y[0] * 0).to(torch.int64))
        ga.capture_end()
    with torch.cuda.stream(sb):
        gb.capture_begin()
        out.copy_(landing)
        gb.capture_end()
    ep_a = torch.zeros(1, dtype=torch.int64, device=dev)
    ep_b = torch.zeros(1, dtype=torch.int64, device=dev)
    flags = nat.uncached_zeros((1,), torch.int32, dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    pieces = torch.zeros(1, dtype=torch.int32, device=dev)
    table = torch.tensor([payload.data_ptr(), landing.data_ptr(), n * 8, flags.data_ptr(),
                          pieces.data_ptr()], dtype=torch.int64, device=dev)

    def chain(kinds, child, p0, p1, p2, i0, i64):
        k = len(kinds)
        arr = lambda ty, xs: (ty * k)(*xs)  # noqa: E731
        g, ex = ctypes.c_void_p(), ctypes.c_void_p()
        rc = nat.lib().mx_graph_build_chain(
            k, arr(ctypes.c_int, kinds), arr(ctypes.c_void_p, child), arr(ctypes.c_void_p, p0),
            arr(ctypes.c_void_p, p1), arr(ctypes.c_void_p, p2), arr(ctypes.c_int, i0),
            arr(ctypes.c_int64, i64), ctypes.byref(g), ctypes.byref(ex))
        assert rc == 0, rc
        return g, ex

    A = chain([5, 0, 6], [0, ga.raw_cuda_graph(), 0], [ep_a.data_ptr(), 0, table.data_ptr()],
              [0, 0, ep_a.data_ptr()], [0, 0, 0], [0, 0, 1], [0, 0, n * 8])
    B = chain([5, 7, 0], [0, 0, gb.raw_cuda_graph()], [ep_b.data_ptr(), flags.data_ptr(), 0],
              [0, ep_b.data_ptr(), 0], [0, err.data_ptr(), 0], [0, 1, 0], [0, 0, 0])
    try:
        for r in range(1, 6):
            val.fill_(1000 + r)
            torch.cuda.synchronize()
            nat.check(nat.lib().mx_graph_launch(B[1], sb.cuda_stream), "launch B")
            nat.check(nat.lib().mx_graph_launch(A[1], sa.cuda_stream), "launch A")
            torch.cuda.synchronize()
            assert int(err.item()) == 0, f"replay {r}: the flag wait timed out"
            assert int(flags.item()) == r and int(ep_a.item()) == r and int(ep_b.item()) == r
            assert bool((out == 1000 + r).all()), (r, out[:4].tolist())
    finally:
        for g, ex in (A, B):
            nat.lib().mx_graph_free(g, ex)
    print("flag: 5 replays ordered")


def replay_case():
    import warnings

    from moose_amd.runtime.local import LocalMooseRuntime
    from test_spmd import _args
    from test_spmd import _comp

    os.environ["MOOSEX_PARTY_STREAMS"] = "1"
    ids = ["alice", "bob", "carole"]
    comp, args = _comp(False), _args()
    devs = {i: "cuda:0" for i in ids}
    want = LocalMooseRuntime(ids, device_map=devs, seed=11, use_graphs=False
                             ).evaluate_computation(comp, args)
    rt = LocalMooseRuntime(ids, device_map=devs, seed=11, use_graphs=True)
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)  # a fallback fails the case
        for _ in range(5):
            got = rt.evaluate_computation(comp, args)
            assert set(got) == set(want)
            for k in want:
                assert np.array_equal(np.asarray(got[k]), np.asarray(want[k])), k
    (_, tapes), = rt._party_tapes.values()
    assert tapes is not False and tapes.replay_form == "party_graphs", tapes.fallback
    assert tapes.validated is True and tapes.fallback is None
    assert rt.last_replay == {"form": "party_graphs", "validated": True, "fallback": None}
    assert tapes.tapes[0].replays == 3
    print("replay: validated, 3 replays bitwise equal to eager")


def fault_case():
    """MOOSEX_FAULT=party_landing: the first push writes a scratch buffer instead of its
    receiver's landing buffer.  With the streams on queues of their own the flags all
    arrive, so the capture-time validation must catch the wrong VALUES."""
    import warnings

    from moose_amd.runtime.local import LocalMooseRuntime
    from test_spmd import _args
    from test_spmd import _comp

    os.environ["MOOSEX_PARTY_STREAMS"] = "1"
    os.environ["MOOSEX_FAULT"] = "party_landing"
    ids = ["alice", "bob", "carole"]
    comp, args = _comp(False), _args()
    devs = {i: "cuda:0" for i in ids}
    want = LocalMooseRuntime(ids, device_map=devs, seed=11, use_graphs=False
                             ).evaluate_computation(comp, args)
    rt = LocalMooseRuntime(ids, device_map=devs, seed=11, use_graphs=True)
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        for _ in range(4):
            got = rt.evaluate_computation(comp, args)
            for k in want:
                assert np.array_equal(np.asarray(got[k]), np.asarray(want[k])), k
    (_, tapes), = rt._party_tapes.values()
    assert tapes.validated is False and tapes.replay_form == "per_action"
    assert "differ from the per-action replay" in tapes.fallback, tapes.fallback
    assert any("failed validation" in str(w.message) for w in caught)
    assert rt.last_replay["form"] == "per_action" and tapes.tapes[0].replays == 2
    print("fault: caught by validation ->", tapes.fallback)


def fallback_case():
    """A per-party stream replay that reports a lost message (TransportError) AFTER the
    validation passed is redone -- and every later replay runs -- per action, bitwise equal
    to eager."""
    import warnings

    from moose_amd.parallel import threads as T
    from moose_amd.parallel.transport import TransportError
    from moose_amd.runtime.local import LocalMooseRuntime
    from test_spmd import _args
    from test_spmd import _comp

    os.environ["MOOSEX_PARTY_STREAMS"] = "1"
    ids = ["alice", "bob", "carole"]
    comp, args = _comp(False), _args()
    devs = {i: "cuda:0" for i in ids}
    want = LocalMooseRuntime(ids, device_map=devs, seed=11, use_graphs=False
                             ).evaluate_computation(comp, args)
    calls = {"n": 0}
    orig = T.PartyTapes._replay_streams

    def flaky(self, arguments):
        calls["n"] += 1
        if calls["n"] == 3:  # 1: the validation, 2: the first replay, 3: the second
            raise TransportError("injected: a message never arrived")
        return orig(self, arguments)

    T.PartyTapes._replay_streams = flaky
    rt = LocalMooseRuntime(ids, device_map=devs, seed=11, use_graphs=True)
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        for _ in range(6):
            got = rt.evaluate_computation(comp, args)
            for k in want:
                assert np.array_equal(np.asarray(got[k]), np.asarray(want[k])), k
    assert any("stream graphs disabled" in str(w.message) for w in caught)
    (_, tapes), = rt._party_tapes.values()
    assert tapes.validated is True and tapes._party_graphs is None and calls["n"] == 3
    print("fallback: per-action after the injected loss")


if __name__ == "__main__":
    {"flag": flag_case, "replay": replay_case, "fault": fault_case,
     "fallback": fallback_case}[sys.argv[1]]()
