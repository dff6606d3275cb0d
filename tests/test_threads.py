"""Parties as threads of one process, each on its own device (``LocalMooseRuntime(...,
device_map=...)``, parallel/threads.py; VERDICT r3 "what's missing" 5: single-process
multi-GPU LocalMooseRuntime).  CPU: every party on the host; GPU: every party on its own
HIP stream of cuda:0, and on three GPUs when the box has them."""
import numpy as np
import pytest
import torch

import moose_amd as pm
from moose_amd.parallel import threads as T
from moose_amd.runtime.local import LocalMooseRuntime

from test_spmd import _args
from test_spmd import _comp

IDS = ["alice", "bob", "carole"]


def _check_against_stacked(dev_map, outsider=False):
    comp = _comp(outsider)
    idents = IDS + (["dave"] if outsider else [])
    args = _args()
    want = LocalMooseRuntime(idents, device="cpu").evaluate_computation(comp, args)
    rt = LocalMooseRuntime(idents, device_map={i: dev_map(k) for k, i in enumerate(idents)},
                           timeout=300)
    got = rt.evaluate_computation(comp, args)
    assert set(got) == set(want)
    for k in want:
        np.testing.assert_allclose(np.asarray(got[k], dtype=np.float64),
                                   np.asarray(want[k], dtype=np.float64), atol=2e-4)
    assert set(rt.last_timings) == set(idents)
    assert rt.last_stats.rounds > 0
    return rt


@pytest.mark.parametrize("outsider", [False, True])
def test_thread_parties_match_stacked_cpu(outsider):
    _check_against_stacked(lambda k: "cpu", outsider)


def test_thread_parties_lr_inference_rounds_cpu():
    """The tutorial LR inference with the parties as threads: the per-party protocol's
    round count (scripts/lr_rounds.py --layout party) and the model's probabilities."""
    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial

    tm = logistic_regression_tutorial(128)
    rt = LocalMooseRuntime(IDS, device_map={i: "cpu" for i in IDS}, timeout=300)
    for _ in range(2):
        got = list(rt.evaluate_computation(tm.computation, {"x": tm.x_test}).values())[0]
        assert np.abs(got - tm.proba).max() < 1e-3
    rounds = {i: s.rounds for i, s in rt.last_stats_by_identity.items()}
    assert len(set(rounds.values())) == 1 and rounds["alice"] <= 46, rounds


def test_thread_parties_lowered_graph_cpu():
    from moose_amd.compiler import passes

    comp = _comp(False)
    args = _args()
    want = LocalMooseRuntime(IDS, device="cpu").evaluate_computation(comp, args)
    rt = LocalMooseRuntime(IDS, device_map={i: "cpu" for i in IDS}, timeout=300)
    got = rt.evaluate_computation(comp, args, compiler_passes=passes.DEFAULT_PASSES)
    assert set(got) == set(want)
    for k in want:
        np.testing.assert_allclose(np.asarray(got[k], dtype=np.float64),
                                   np.asarray(want[k], dtype=np.float64), atol=1e-5)


def test_thread_party_failure_raises_instead_of_hanging():
    """One party fails (a Load of a key only its storage lacks); the others are blocked on
    its messages and must raise too, so the evaluation ends with the cause."""
    alice, bob, carole = (pm.host_placement(n) for n in IDS)
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])

    @pm.computation
    def g():
        with bob:
            x = pm.load("x", dtype=pm.float64)
            xf = pm.cast(x, dtype=pm.fixed(14, 23))
        with rep:
            y = pm.mul(xf, xf)
        with carole:
            return pm.cast(y, dtype=pm.float64)

    rt = LocalMooseRuntime(IDS, device_map={i: "cpu" for i in IDS}, timeout=60)
    with pytest.raises(Exception) as ei:
        rt.evaluate_computation(g, {})
    assert "x" in str(ei.value) and "TransportError" not in type(ei.value).__name__
    rt.write_value_to_storage("bob", "x", np.array([1.5, -2.0]))
    out = list(rt.evaluate_computation(g, {}).values())[0]
    np.testing.assert_allclose(out, [2.25, 4.0], atol=1e-5)


def test_receive_from_a_finished_party_raises_at_once():
    """a party that returns without sending what its peer expects (a protocol
    desynchronisation) must not leave the peer polling forever -- with no timeout set the
    receive raises as soon as the sender's thread has finished and its mailbox is empty."""
    import time

    from moose_amd.parallel.threads import Hub
    from moose_amd.parallel.threads import ThreadTransport
    from moose_amd.parallel.transport import TransportError

    hub = Hub(["cpu", "cpu"], timeout=None)
    a, b = ThreadTransport(0, hub), ThreadTransport(1, hub)
    b.send(torch.arange(3), 0)  # one message, then party 1 returns
    hub.finish(1)
    assert torch.equal(a.recv(1), torch.arange(3))  # what was sent still arrives
    t0 = time.perf_counter()
    with pytest.raises(TransportError, match="finished without sending"):
        a.recv(1)
    assert time.perf_counter() - t0 < 5
    assert hub.failed is not None


def test_mailbox_routes_a_message_in_place_on_the_second_capture():
    """threads.Mailbox: the first capture learns that party 0's first outbox buffer became
    its first message to party 1; the second capture hands party 0 a persistent buffer for
    it and lands party 1's receive in that same buffer (no copy).  An outbox buffer that is
    never sent is not routed (the transport declines it the second time)."""
    from moose_amd.parallel.transport import CommStep

    mb = T.Mailbox()

    def capture():
        steps = {0: [], 1: []}
        trs = [T.ThreadTransport(i, None, device="cpu", world=2) for i in range(2)]
        for i, tr in enumerate(trs):
            tr.mailbox = mb
            tr.tape = steps[i].append
            tr.log = {1 - i: [("t", (2, 2), torch.int64, None)]}
        msg = trs[0].outbox((2, 2), torch.int64)
        kept = trs[0].outbox((3,), torch.int64)  # this party's own: never sent
        trs[0].exchange([(msg, 1)], [])
        got = torch.empty((2, 2), dtype=torch.int64)
        trs[1].exchange([], [(got, 0)])
        return msg, kept, got, steps

    msg, kept, got, steps = capture()
    assert mb.route == {(0, 1, 0): 0}
    assert got.data_ptr() != msg.data_ptr()  # pass 1: the receive is a copy target
    mb.prepare("cpu")
    msg, kept, got, steps = capture()
    assert got.data_ptr() == msg.data_ptr() == mb.slots[(0, 0)].data_ptr()
    assert kept is None and (0, 1) not in mb.slots  # the session allocates it as usual
    (step,), = [steps[1]]
    assert isinstance(step, CommStep) and step.recvs[0][0].data_ptr() == msg.data_ptr()


def test_device_map_rejects_unknown_identity():
    with pytest.raises(ValueError):
        LocalMooseRuntime(IDS, device_map={"mallory": "cpu"})


@pytest.mark.gpu
def test_thread_parties_on_gpu_streams():
    """Every party on its own HIP stream of cuda:0 (the one-GPU box), then one party per GPU
    when three are visible: results equal the stacked session's within TruncPr rounding."""
    _check_against_stacked(lambda k: "cuda:0")
    n = torch.cuda.device_count()
    if n >= 3:
        _check_against_stacked(lambda k: f"cuda:{k % n}")


@pytest.mark.gpu
def test_thread_parties_lr_inference_gpu(monkeypatch):
    """The tutorial LR inference with each party a thread on its own stream (and GPU when
    three are visible): the second evaluation records per-party tapes, later ones replay
    them from one host thread (PartyTapes).  Prints eager and replay p50."""
    import time

    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial

    monkeypatch.setenv("MOOSEX_GRAPHS_DEBUG", "1")  # a capture failure fails the test
    tm = logistic_regression_tutorial(128)
    n = torch.cuda.device_count()
    devs = {i: f"cuda:{k % n if n >= 3 else 0}" for k, i in enumerate(IDS)}
    lat = {}
    for mode in (False, True):
        rt = LocalMooseRuntime(IDS, device_map=devs, timeout=120, use_graphs=mode)
        ts = []
        for _ in range(8):
            t0 = time.perf_counter()
            got = list(rt.evaluate_computation(tm.computation, {"x": tm.x_test}).values())[0]
            ts.append(time.perf_counter() - t0)
            assert np.abs(got - tm.proba).max() < 1e-3
        lat[mode] = sorted(ts[3:])[2] * 1e3
        if mode:
            (comp, tapes), = rt._party_tapes.values()
            assert tapes is not False and tapes.tapes[0].replays >= 5
            issue = sorted(tapes.issue_s)[len(tapes.issue_s) // 2] * 1e3
    print(f"thread parties LR inference ({min(n, 3)} GPU): eager p50 {lat[False]:.2f} ms, "
          f"replay p50 {lat[True]:.3f} ms (host issue {issue:.3f} ms), "
          f"rounds {rt.last_stats.rounds}")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["serial", "copied-messages", "unbatched-launches",
                                  "copy-per-message", "per-action", "streams"])
def test_thread_party_tapes_replay_bitwise_equal_eager(mode, monkeypatch):
    """Seeded sessions: a replay re-draws the seeded keys as a fresh eager evaluation does,
    so every replay's outputs equal the eager ones bitwise (parties on cuda:0): the tapes
    composed into one hipGraph in a round-synchronous total order (default on one device:
    each round's messages one batched copy kernel, or one copy node per message; the same
    launch of several parties between two rounds one party-batched node, csrc/
    party_batch.h, or one node per launch; the jobs tails' messages read where their
    senders wrote them, threads.Mailbox, or copied), and the per-action replay."""
    if mode == "streams":
        # per-party stream graphs need their streams on distinct hardware queues: a fresh
        # child process with enough queues (tests/gpu_streams_child.py) -- no skip
        _streams_child("replay")
        return
    composed = mode not in ("per-action", "streams")
    monkeypatch.setenv("MOOSEX_PARTY_GRAPH", "1" if composed else "0")
    monkeypatch.setenv("MOOSEX_PARTY_COPY_BATCH", "0" if mode == "copy-per-message" else "1")
    monkeypatch.setenv("MOOSEX_PARTY_STREAMS", "1" if mode == "streams" else "0")
    monkeypatch.setattr(T, "MERGE_PARTIES", mode != "unbatched-launches")
    monkeypatch.setattr(T, "INPLACE", mode != "copied-messages")
    comp = _comp(False)
    args = _args()
    devs = {i: "cuda:0" for i in IDS}
    eager = LocalMooseRuntime(IDS, device_map=devs, seed=11, use_graphs=False)
    want = eager.evaluate_computation(comp, args)
    rt = LocalMooseRuntime(IDS, device_map=devs, seed=11, use_graphs=True)
    import warnings

    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        for _ in range(4):
            got = rt.evaluate_computation(comp, args)
            assert set(got) == set(want)
            for k in want:
                assert np.array_equal(np.asarray(got[k]), np.asarray(want[k])), k
    assert not any("stream graphs" in str(w.message) for w in caught)
    (c, tapes), = rt._party_tapes.values()
    assert tapes is not False and tapes.tapes[0].replays == 2
    assert (tapes._composed is not None) == composed
    assert (tapes._party_graphs is not None) == (mode == "streams")
    if mode == "serial":  # the parties' protocol launches batched into shared nodes
        assert tapes.graph_nodes["merged_away"] > 0, tapes.graph_nodes
        assert tapes.graph_nodes["inplace_messages"] > 0, tapes.graph_nodes
    if mode == "copied-messages":
        assert tapes.inplace_messages == 0


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["output", "input"])
def test_composed_replay_with_an_outsider_bitwise_equal_eager(where):
    """Four in-process parties on cuda:0 and dave outside the replicated placement, who
    receives an output or OWNS an input (shared with two fresh seeds: key slots the tape
    refreshes at every replay and ships as slot images).  The composed replay keeps the
    fourth party's segments unbatched and in order, and every replay equals the eager
    seeded evaluation bitwise."""
    if where == "input":
        _replay_equals_eager(_comp(True), IDS + ["dave"], _args())
        return
    alice, bob, carole, dave = (pm.host_placement(n) for n in IDS + ["dave"])
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])
    fp = pm.fixed(14, 23)

    @pm.computation
    def comp(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64)),
             y: pm.Argument(placement=bob, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=fp)
        with bob:
            yf = pm.cast(y, dtype=fp)
        with rep:
            z = pm.dot(xf, yf)
            s = pm.sigmoid(z)
        with dave:
            return pm.cast(s, dtype=pm.float64), pm.cast(z, dtype=pm.float64)

    _replay_equals_eager(comp, IDS + ["dave"], _args())


def _replay_equals_eager(comp, idents, args):
    devs = {i: "cuda:0" for i in idents}
    want = LocalMooseRuntime(idents, device_map=devs, seed=5,
                             use_graphs=False).evaluate_computation(comp, args)
    rt = LocalMooseRuntime(idents, device_map=devs, seed=5, use_graphs=True)
    for _ in range(4):
        got = rt.evaluate_computation(comp, args)
        assert set(got) == set(want)
        for k in want:
            assert np.array_equal(np.asarray(got[k]), np.asarray(want[k])), k
    (_, tapes), = rt._party_tapes.values()
    assert tapes is not False and tapes.replay_form == "composed"
    assert tapes.tapes[0].replays >= 2


def test_party_tapes_schedule_pairs_rounds():
    """The replay order of PartyTapes (CPU, mock tapes): a ring shift, then a dealer's
    send-only round to two receive-only parties.  Every receive is issued after its
    matched send's event, every party's steps stay in order, and an unmatched receive is
    a capture error (the evaluation then stays eager)."""
    from moose_amd.parallel.threads import PartyTapes
    from moose_amd.parallel.transport import CommStep
    from moose_amd.runtime.graphs import CaptureError

    class _T:
        def __init__(self, steps):
            self.steps = steps

    def e(n):
        return torch.zeros(n)

    tapes = [
        ["a0", CommStep([(e(2), 1)], [(e(2), 2)]), "a1", CommStep([], [(e(3), 2)]), "a2"],
        ["b0", CommStep([(e(2), 2)], [(e(2), 0)]), CommStep([], [(e(3), 2)]), "b1"],
        ["c0", CommStep([(e(2), 0)], [(e(2), 1)]), "c1", CommStep([(e(3), 0), (e(3), 1)], [])],
    ]
    pt = PartyTapes.__new__(PartyTapes)
    pt.tapes = [_T(s) for s in tapes]
    acts = pt._schedule()
    order = {p: [a[2] for a in acts if a[0] == "g" and a[1] == p] for p in range(3)}
    assert order == {0: ["a0", "a1", "a2"], 1: ["b0", "b1"], 2: ["c0", "c1"]}
    recorded = set()
    for a in acts:
        if a[0] == "rec":
            recorded.add(id(a[2]))
        elif a[0] == "cp":
            assert id(a[5]) in recorded  # the send's event was recorded before
    assert sum(a[0] == "cp" for a in acts) == 5
    pt.tapes = [_T([CommStep([], [(e(1), 1)])]), _T(["x"])]
    with pytest.raises(CaptureError):
        pt._schedule()


def test_party_tapes_round_schedule_batches_messages():
    """The composed one-GPU order (PartyTapes._schedule_rounds, CPU mock tapes): every
    party's segments stay in program order, each message is copied after its sender's
    segment that produced it and before its receiver's next segment, and the messages of
    one round of all parties form ONE batch."""
    from moose_amd.parallel.threads import PartyTapes
    from moose_amd.parallel.transport import CommStep
    from moose_amd.runtime.graphs import CaptureError

    class _T:
        def __init__(self, steps):
            self.steps = steps

    def e(n):
        return torch.zeros(n)

    # round 1: a ring shift (3 messages); round 2: the dealer's two messages
    tapes = [
        ["a0", CommStep([(e(2), 1)], [(e(2), 2)]), "a1", CommStep([], [(e(3), 2)]), "a2"],
        ["b0", CommStep([(e(2), 2)], [(e(2), 0)]), CommStep([], [(e(3), 2)]), "b1"],
        ["c0", CommStep([(e(2), 0)], [(e(2), 1)]), "c1", CommStep([(e(3), 0), (e(3), 1)], [])],
    ]
    pt = PartyTapes.__new__(PartyTapes)
    pt.tapes = [_T(s) for s in tapes]
    acts = pt._schedule_rounds()
    order = {p: [a[2] for a in acts if a[0] == "g" and a[1] == p] for p in range(3)}
    assert order == {0: ["a0", "a1", "a2"], 1: ["b0", "b1"], 2: ["c0", "c1"]}
    batches = [a[1] for a in acts if a[0] == "cpb"]
    assert [len(b) for b in batches] == [3, 2]
    pos = {a[2]: i for i, a in enumerate(acts) if a[0] == "g"}
    first = acts.index(("cpb", batches[0]))
    second = acts.index(("cpb", batches[1]))
    assert max(pos["a0"], pos["b0"], pos["c0"]) < first < min(pos["a1"], pos["b1"], pos["c1"])
    assert pos["c1"] < second < min(pos["a2"], pos["b1"])
    assert {(r, s) for r, s, _, _ in batches[1]} == {(0, 2), (1, 2)}
    pt.tapes = [_T([CommStep([], [(e(1), 1)])]), _T(["x"])]
    with pytest.raises(CaptureError):
        pt._schedule_rounds()


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_party_ks_chain_matches_per_level(dev, monkeypatch):
    """SPMDSession.p_ks_chain (each level's xor folded into the next level's cross-term
    kernel, the last xor into the sum kernel) gives bitwise the outputs of the per-level
    path (p_ks_level + share-wise sum), seeded, with the same round count."""
    comp = _comp(False)
    args = _args()
    outs = {}
    for chain in ("1", "0"):
        monkeypatch.setenv("MOOSEX_KS_CHAIN", chain)
        rt = LocalMooseRuntime(IDS, device_map={i: dev for i in IDS}, seed=5, timeout=300,
                               use_graphs=False)
        outs[chain] = (rt.evaluate_computation(comp, args), rt.last_stats.rounds)
    (a, ra), (b, rb) = outs["1"], outs["0"]
    assert ra == rb
    for k in b:
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k


@pytest.mark.gpu
def test_device_flag_push_wait_orders_two_streams():
    """The per-party stream graphs' message signalling alone (csrc/party_graph.hip k_push /
    k_wait under mx_graph_build_chain): graph A delays (a chain of kernels), writes a payload
    and pushes it to an uncached landing buffer with a flag; graph B, launched FIRST on
    another stream, waits for the flag and copies the landing buffer out.  Every replay B
    must see A's payload of that replay.  Run in a fresh child process whose two streams
    have hardware queues of their own (tests/gpu_streams_child.py): a timed-out wait FAILS."""
    _streams_child("flag")


def _streams_child(case):
    import os
    import subprocess
    import sys

    env = dict(os.environ, GPU_MAX_HW_QUEUES="16", PYTHONUNBUFFERED="1")
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "gpu_streams_child.py"), case],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-4000:], r.stderr[-4000:])


@pytest.mark.gpu
def test_party_streams_validation_catches_a_corrupted_landing_buffer():
    """MOOSEX_FAULT=party_landing: the first message's push writes a scratch buffer, so its
    receiver reads a stale landing buffer.  The capture-time validation (the per-party
    graphs against the per-action replay of the same tapes and keys) catches the wrong
    values, records the failure and keeps the per-action replay, bitwise equal to eager
    (tests/gpu_streams_child.py fault: streams on queues of their own, so the flags all
    arrive and only the values can give it away)."""
    _streams_child("fault")


@pytest.mark.gpu
def test_party_streams_fall_back_to_per_action_replay():
    """A per-party stream replay that reports a lost message (TransportError) after the
    capture-time validation passed is redone -- and every later replay runs -- with the
    per-action replay of the same tapes, still bitwise equal to eager
    (tests/gpu_streams_child.py fallback)."""
    _streams_child("fallback")


def test_shared_constant_caches_first_in_wins():
    """Parties on threads may make one constant at once: the shared caches keep the first
    (an entry keyed by an object's id must keep that object alive), so a dropped second
    copy's id can never alias a cached constant later."""
    from moose_amd.ops import ring as R

    cache = {}
    a, b = R.fill((3,), 1, 64, "cpu"), R.fill((3,), 1, 64, "cpu")
    R._cache_put(cache, "k", a, 10)
    R._cache_put(cache, "k", b, 10)
    assert cache["k"] is a


@pytest.mark.gpu
def test_encoded_constant_cache_checks_identity():
    """An encoded-constant entry is only returned for the very tensor it was made from (a
    freed constant's id may come back as another tensor's: the round-5 intermittent
    'dot shape mismatch' of threaded parties on one GPU)."""
    from moose_amd.ops import ring as R

    x = torch.ones(3, 2, dtype=torch.float64, device="cuda:0")
    y = torch.full((200, 10), 2.0, dtype=torch.float64, device="cuda:0")
    R.CONST_IDS.add(id(y))
    R._ENCODED_CONSTS[(id(y), 10, 128)] = (x, R.encode(x, 10, 128))  # a stale entry
    try:
        e = R.encode_lazy(y, 10, 128)
        assert tuple(e.shape) == (200, 10)
        assert np.allclose(R.decode(e, 10).cpu().numpy(), 2.0)
    finally:
        R.CONST_IDS.discard(id(y))
        R._ENCODED_CONSTS.pop((id(y), 10, 128), None)


@pytest.mark.gpu
def test_party_tapes_capture_a_large_product():
    """A taped product large enough for the CRT GEMM (its per-stream workspace grows while
    the tape's own stream is capturing: the allocation runs in relaxed capture mode) is
    recorded and replayed -- before, the capture failed and the next eager evaluation hit
    'operation not permitted when stream is capturing'."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "benchmarks"))
    from dot_product import build

    from moose_amd.runtime.local import to_native

    native = to_native(build("seq", 1))
    n = 512
    args = {"x_arg": np.ones((n, n)), "y_arg": np.identity(n)}
    rt = LocalMooseRuntime(IDS, device_map={i: "cuda:0" for i in IDS}, use_graphs=True,
                           timeout=120)
    for _ in range(4):
        out = rt.evaluate_computation(native, args)
        np.testing.assert_allclose(np.asarray(next(iter(out.values()))), args["x_arg"],
                                   atol=1e-6)
    (_, tapes), = rt._party_tapes.values()
    assert tapes is not False and all(t.replays >= 1 for t in tapes.tapes)


def test_composed_schedule_chunks_keep_order_and_bound_segments():
    """PartyTapes._compose splits the composed total order into executables of at most N
    segments (threads.chunk_bounds): consecutive, covering every node once, copies kept
    with the segments before them."""
    from moose_amd.parallel.threads import chunk_bounds

    kinds = [0, 2, 0, 0, 1, 2, 0, 0, 0, 2, 2, 0]
    for per in (1, 2, 3, 5, 100):
        b = chunk_bounds(kinds, per)
        assert b[0][0] == 0 and b[-1][1] == len(kinds)
        assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
        assert all(sum(k == 0 for k in kinds[s:e]) <= per for s, e in b)
        assert all(kinds[s] == 0 for s, _ in b[1:])  # a new chunk starts at a segment
    assert chunk_bounds(kinds, 100) == [(0, len(kinds))]


@pytest.mark.gpu
def test_large_party_tape_composes_into_one_flat_executable():
    """A 40-iteration LogReg training tape of the parties (hundreds of segments): composed
    into ONE executable with every kernel-only segment flattened (no 200-segment chunks, no
    256-segment cap -- the round-5 crash was the flattening of captured copy nodes,
    profiles/r6_graph_flatten_segfault.md), and its seeded replays bitwise equal to eager."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "benchmarks"))
    from logreg_train import build_training

    from moose_amd.runtime.local import to_native

    native = to_native(build_training(16, 40, n_features=8))
    rng = np.random.default_rng(0)
    args = {"x": rng.standard_normal((640, 8)), "y": rng.integers(2, size=(640, 1)) * 1.0,
            "w_0": np.zeros((8, 1)), "b_0": np.zeros((1, 1))}
    devs = {i: "cuda:0" for i in IDS}
    want = LocalMooseRuntime(IDS, device_map=devs, seed=5, use_graphs=False,
                             timeout=300).evaluate_computation(native, args)
    rt = LocalMooseRuntime(IDS, device_map=devs, seed=5, use_graphs=True, timeout=300)
    for _ in range(4):
        got = rt.evaluate_computation(native, args)
        for k in want:
            assert np.array_equal(np.asarray(got[k]), np.asarray(want[k])), k
    (_, tapes), = rt._party_tapes.values()
    assert tapes is not False and tapes.replay_form == "composed"
    assert tapes.segments > 256 and tapes.graph_nodes["executables"] == 1, tapes.graph_nodes
    assert tapes.tapes[0].replays == 2
