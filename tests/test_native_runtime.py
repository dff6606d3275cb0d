"""Native runtime core (csrc/runtime via ``_moosert``): parser, graph passes, mailbox,
TCP networking and the dataflow scheduler -- each checked against the pure-Python
implementation it replaces or against the plaintext result.

Reference parity: textual/parsing.rs (parser), computation.rs:1879-1942 + toposort.rs +
pruning.rs (graph), networking/local.rs (exactly-once rendezvous), tcpstream.rs (TCP),
execution/asynchronous.rs (dataflow, first-error abort)."""
import glob
import os
import threading

import numpy as np
import pytest

from moose_amd.compiler import passes
from moose_amd.ir import textual
from moose_amd.ir.computation import Computation
from moose_amd.runtime import native_rt as N
from moose_amd.runtime.dataflow import TcpTransport
from moose_amd.runtime.graph_executor import GraphExecutionError
from moose_amd.runtime.graph_executor import GraphExecutor

REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NETWORKED = os.path.join(REF, "tutorials", "dotprod-networked.moose")


def _moose_files():
    files = sorted(glob.glob(os.path.join(REPO, "examples", "*.moose")))
    files += sorted(glob.glob(os.path.join(REF, "tutorials", "*.moose")))
    files += sorted(glob.glob(os.path.join(REF, "examples", "*.moose")))
    return files


def test_extension_loads():
    m = N.mod()
    assert m.__file__.startswith(os.path.join(REPO, "moose_amd", "_native"))
    assert N.enabled()


@pytest.mark.parametrize("path", _moose_files())
def test_native_parser_matches_python_parser(path):
    src = open(path).read()
    a = textual.parse_computation_py(src, parallel=False)
    b = N.parse(src, threads=4)
    assert a.to_textual() == b.to_textual()


def test_parallel_native_parse_of_large_graph():
    path = os.path.join(REF, "moose", "benches", "rep_computation.moose")
    if not os.path.exists(path):
        pytest.skip("reference checkout not available")
    src = open(path).read()
    one = N.parse(src, threads=1)
    many = N.parse(src, threads=8)
    assert len(one) == len(many) == 19045
    assert one.to_textual() == many.to_textual()


def test_parse_errors_are_parse_errors():
    with pytest.raises(textual.ParseError, match="unknown operator"):
        textual.parse_computation("x = NotAnOp: () -> HostUnit () @Host(alice)")
    with pytest.raises(textual.ParseError, match="owners"):
        textual.parse_computation(
            "x = Identity: (HostFloat32Tensor) -> HostFloat32Tensor (a) @Replicated(a, b)")


def test_constants_round_trip_exactly():
    big = (1 << 127) + 12345
    src = (f'a = Constant{{value = HostRing128Tensor([[{big}, 1], [2, 3]])}}: () -> '
           f'HostRing128Tensor () @Host(alice)\n'
           'b = Constant{value = Float64(-1.5e-07)}: () -> Float64 () @Host(alice)\n'
           'c = Constant{value = HostString("q\\"x")}: () -> HostString () @Host(alice)\n'
           'd = Constant{value = HostShape([2, 3])}: () -> HostShape () @Host(alice)\n')
    comp = N.parse(src)
    assert comp.operations[0].attrs["value"].value[0, 0] == big
    assert comp.operations[1].attrs["value"].value == -1.5e-07
    assert comp.operations[2].attrs["value"].value == 'q"x'
    assert comp.operations[3].attrs["value"].value == (2, 3)
    assert comp.to_textual() == textual.parse_computation_py(src).to_textual()


@pytest.mark.skipif(not os.path.exists(NETWORKED), reason="reference checkout not available")
def test_native_toposort_matches_python():
    comp = Computation.from_textual(open(NETWORKED).read())
    a = comp.toposorted_py()
    b = N.toposort(comp)
    assert [op.name for op in a.operations] == [op.name for op in b.operations]
    assert N.graph_of(b).first_out_of_order() == -1


def test_graph_detects_cycles_and_unknown_inputs():
    cyc = Computation.from_textual(
        "a = Identity: (HostFloat64Tensor) -> HostFloat64Tensor (b) @Host(x)\n"
        "b = Identity: (HostFloat64Tensor) -> HostFloat64Tensor (a) @Host(x)\n")
    with pytest.raises(ValueError, match="cycle"):
        cyc.toposorted()
    bad = Computation.from_textual(
        "a = Identity: (HostFloat64Tensor) -> HostFloat64Tensor (zz) @Host(x)\n")
    with pytest.raises(KeyError):
        bad.toposorted()


@pytest.mark.skipif(not os.path.exists(NETWORKED), reason="reference checkout not available")
def test_prune_keeps_send_receive_pairs_and_stats():
    comp = Computation.from_textual(open(NETWORKED).read())
    pruned = passes.prune(comp)
    kinds = [op.kind for op in pruned.operations]
    assert kinds.count("Send") == kinds.count("Receive") == 25
    st = N.stats(comp)
    assert st["ops"] == 167 and st["op_histogram"]["Send"] == 25
    assert st["comm_rounds"] >= 2 and st["depth"] > st["comm_rounds"]


def test_mailbox_exactly_once_and_timeout():
    mb = N.mod().Mailbox()
    mb.put("s/1", "alice", b"abc")
    with pytest.raises(RuntimeError, match="duplicate"):
        mb.put("s/1", "alice", b"abc")
    assert mb.take("s/1", 1.0) == ("alice", b"abc")
    with pytest.raises(RuntimeError, match="already received"):
        mb.take("s/1", 0.05)
    with pytest.raises(N.mod().NativeNetTimeout):
        mb.take("s/2", 0.05)


def test_dataflow_runs_every_op_once_in_dependency_order():
    comp = Computation.from_textual(
        "a = Constant{value = HostFloat64Tensor([1.0])}: () -> HostFloat64Tensor () @Host(x)\n"
        "b = Identity: (HostFloat64Tensor) -> HostFloat64Tensor (a) @Host(x)\n"
        "c = Identity: (HostFloat64Tensor) -> HostFloat64Tensor (a) @Host(x)\n"
        "d = Add: (HostFloat64Tensor, HostFloat64Tensor) -> HostFloat64Tensor (b, c) @Host(x)\n")
    g = N.graph_of(comp)
    seen, lock = [], threading.Lock()

    def cb(i):
        with lock:
            for p in g.preds(i):
                assert p in seen
            seen.append(i)

    st = N.mod().Dataflow(g, [0, 1, 2, 3], [""] * 4).run(cb, 3)
    assert sorted(seen) == [0, 1, 2, 3] and st["ops_run"] == 4


def test_dataflow_first_error_aborts():
    comp = Computation.from_textual(
        "a = Constant{value = HostFloat64Tensor([1.0])}: () -> HostFloat64Tensor () @Host(x)\n"
        "b = Identity: (HostFloat64Tensor) -> HostFloat64Tensor (a) @Host(x)\n")
    g = N.graph_of(comp)
    ran = []

    def cb(i):
        ran.append(i)
        raise ZeroDivisionError("boom")

    with pytest.raises(ZeroDivisionError, match="boom"):
        N.mod().Dataflow(g, [0, 1], ["", ""]).run(cb, 2)
    assert ran == [0]


def test_dataflow_deadline_on_missing_message():
    comp = Computation.from_textual(
        'r = Receive{rendezvous_key = 01, sender = "y"}: () -> HostFloat64Tensor () @Host(x)\n')
    mb = N.mod().Mailbox()
    with pytest.raises(N.mod().NativeNetTimeout, match="deadline"):
        N.mod().Dataflow(N.graph_of(comp), [0], ["k"], mb).run(lambda i: None, 1, 0.2)


@pytest.mark.skipif(not os.path.exists(NETWORKED), reason="reference checkout not available")
def test_local_dataflow_runs_networked_tutorial():
    comp = Computation.from_textual(open(NETWORKED).read())
    ex = GraphExecutor("cpu", workers=2)
    out = ex.run(comp, {})
    np.testing.assert_allclose(np.asarray(out["output_0"]), [[32.0]], atol=1e-5)
    assert ex.last_run_stats["ops_run"] == 167


def test_duplicate_send_and_orphan_receive_rejected():
    dup = """
a = Constant{value = HostFloat64Tensor([1.0])}: () -> HostFloat64Tensor () @Host(alice)
s1 = Send{rendezvous_key = 01, receiver = "bob"}: (HostFloat64Tensor) -> HostUnit (a) @Host(alice)
s2 = Send{rendezvous_key = 01, receiver = "bob"}: (HostFloat64Tensor) -> HostUnit (a) @Host(alice)
r = Receive{rendezvous_key = 01, sender = "alice"}: () -> HostFloat64Tensor () @Host(bob)
"""
    with pytest.raises(GraphExecutionError, match="duplicate send"):
        GraphExecutor("cpu").run(Computation.from_textual(dup), {})
    orphan = 'r = Receive{rendezvous_key = 02, sender = "alice"}: () -> HostFloat64Tensor () @Host(bob)\n'
    with pytest.raises(GraphExecutionError, match="no Send"):
        GraphExecutor("cpu").run(Computation.from_textual(orphan), {})


def _free_ports(n):
    import socket

    socks = [socket.socket() for _ in range(n)]
    for s in socks:
        s.bind(("127.0.0.1", 0))
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    return ports


def test_tcp_transport_codec_round_trip():
    import torch

    from moose_amd.ops import ring as R

    ports = _free_ports(1)
    tr = TcpTransport("a", {"a": f"127.0.0.1:{ports[0]}"})
    vals = [R.from_ints([[1 << 100, 5]], 128), torch.arange(6.0).reshape(2, 3),
            torch.tensor([True, False]), b"\x00\x01seed", (3, 4), 7, -(1 << 90), 2.5, None, "s"]
    for v in vals:
        w = tr.decode(tr.encode(v), "cpu")
        if isinstance(v, R.RT):
            assert w.bits == 128 and (R.to_ints(w) == R.to_ints(v)).all()
        elif isinstance(v, torch.Tensor):
            assert w.dtype == v.dtype and torch.equal(w, v)
        else:
            assert w == v
    tr.close()


@pytest.mark.skipif(not os.path.exists(NETWORKED), reason="reference checkout not available")
def test_tcp_identities_run_networked_tutorial():
    """Three identities, each with its own executor and TCP endpoint (threads here; the
    vixen CLI runs them as processes), exchange shares by rendezvous key."""
    comp = Computation.from_textual(open(NETWORKED).read())
    ids = ["player0", "player1", "player2"]
    ports = _free_ports(3)
    eps = {r: f"127.0.0.1:{p}" for r, p in zip(ids, ports)}
    results, errors = {}, []

    def party(ident):
        tr = TcpTransport(ident, eps, session_id="t1").start()
        try:
            ex = GraphExecutor("cpu", identity=ident, transport=tr, timeout_s=60)
            results[ident] = (ex.run(comp, {}), tr.stats())
        except Exception as e:  # pragma: no cover - surfaced below
            errors.append((ident, e))
        finally:
            tr.close()

    th = [threading.Thread(target=party, args=(i,)) for i in ids]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors
    np.testing.assert_allclose(np.asarray(results["player2"][0]["output_0"]), [[32.0]], atol=1e-5)
    sent = sum(s["msgs_sent"] for _, st in results.values() for s in st.values())
    assert sent == 25


@pytest.mark.skipif(not os.path.exists(NETWORKED), reason="reference checkout not available")
def test_vixen_tcp_processes_run_networked_tutorial():
    """One OS process per identity (the reference's vixen over raw TCP)."""
    import json
    import subprocess
    import sys

    # the reference's flags: --placement (own identity), --role-assignment, --hosts
    roles = ["player0", "player1", "player2"]
    ids = ["alice", "bob", "carole"]
    ra = json.dumps(dict(zip(roles, ids)))
    hosts = json.dumps({r: f"127.0.0.1:{p}" for r, p in zip(ids, _free_ports(3))})
    env = dict(os.environ, PYTHONPATH=REPO)
    procs = [subprocess.Popen([sys.executable, "-m", "moose_amd.cli.vixen", "--transport", "tcp",
                               "--placement", i, "--role-assignment", ra, "--hosts", hosts,
                               "--comp", NETWORKED, "--timeout", "120"], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for i in ids]
    outs = [p.communicate(timeout=240)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert "[carole] output_0 = [[32.]]" in outs[2]


def _make_certs(d, names):
    """CA + one certificate per name (CN = name) with the openssl CLI."""
    import shutil
    import subprocess

    if shutil.which("openssl") is None:
        pytest.skip("openssl CLI not available")

    def run(*a):
        subprocess.run(["openssl", *a], check=True, capture_output=True, cwd=d)

    run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "ca.key", "-out", "ca.crt",
        "-days", "2", "-subj", "/CN=moosex-test-ca")
    for n in names:
        run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{n}.key", "-out", f"{n}.csr",
            "-subj", f"/CN={n}")
        run("x509", "-req", "-in", f"{n}.csr", "-CA", "ca.crt", "-CAkey", "ca.key",
            "-CAcreateserial", "-out", f"{n}.crt", "-days", "2")
    return str(d)


def _run_parties(comp, ids, eps, certs_for):
    results, errors = {}, []

    def party(ident):
        try:
            tr = TcpTransport(ident, eps, session_id="tls", certs_dir=certs_for(ident),
                              connect_timeout_s=5).start()
        except Exception as e:
            errors.append((ident, e))
            return
        try:
            ex = GraphExecutor("cpu", identity=ident, transport=tr, timeout_s=10)
            results[ident] = ex.run(comp, {})
        except Exception as e:
            errors.append((ident, e))
        finally:
            tr.close()

    th = [threading.Thread(target=party, args=(i,)) for i in ids]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    return results, errors


@pytest.mark.skipif(not os.path.exists(NETWORKED), reason="reference checkout not available")
def test_mutual_tls_networking(tmp_path):
    """mTLS (reference grpc.rs:150-168): authenticated identities run the tutorial; an
    identity whose certificate names someone else cannot join."""
    comp = Computation.from_textual(open(NETWORKED).read())
    ids = ["player0", "player1", "player2"]
    certs = _make_certs(tmp_path, ids + ["mallory"])
    eps = {r: f"127.0.0.1:{p}" for r, p in zip(ids, _free_ports(3))}
    results, errors = _run_parties(comp, ids, eps, lambda i: certs)
    assert not errors, errors
    np.testing.assert_allclose(np.asarray(results["player2"]["output_0"]), [[32.0]], atol=1e-5)

    # player1's endpoint is served with mallory's certificate: nobody may talk to it
    bad = tmp_path / "bad"
    bad.mkdir()
    import shutil

    shutil.copy(tmp_path / "ca.crt", bad / "ca.crt")
    shutil.copy(tmp_path / "mallory.crt", bad / "player1.crt")
    shutil.copy(tmp_path / "mallory.key", bad / "player1.key")
    eps = {r: f"127.0.0.1:{p}" for r, p in zip(ids, _free_ports(3))}
    results, errors = _run_parties(
        comp, ids, eps, lambda i: str(bad) if i == "player1" else certs)
    assert errors and "player2" not in results
    assert any("names 'mallory'" in str(e) or "mismatch" in str(e) or "deadline" in str(e)
               for _, e in errors), errors
