"""Choreographed workers (``comet``/``cometctl``/filesystem sessions) on gloo: sessions
launched through the control-plane store run on long-lived workers (reference
``choreography/grpc.rs`` + ``choreography/filesystem.rs`` behaviour: duplicate session
ids are rejected, results carry per-identity timings, .session files are picked up)."""
import os
import shutil
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IDS = ["alice", "bob", "carole"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _start(port, sessions_dir=None, extra=()):
    env = dict(os.environ, PYTHONPATH=ROOT, WORLD_SIZE="3")
    procs = []
    for r, ident in enumerate(IDS):
        if sessions_dir:  # filesystem choreography worker (rank 0 watches the dir)
            cmd = [sys.executable, "-m", "moose_amd.cli.rudolph", "--identity", ident,
                   "--store", f"127.0.0.1:{port}", "--sessions", sessions_dir,
                   "--backend", "gloo", *extra]
        else:
            cmd = [sys.executable, "-m", "moose_amd.cli.comet", "--identity", ident,
                   "--store", f"127.0.0.1:{port}", "--rank", str(r), "--world", "3",
                   "--backend", "gloo"]
        procs.append(subprocess.Popen(cmd, env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
        if r == 0:
            time.sleep(1.0)  # rank 0 hosts the store
    return procs


def _stop(procs, client):
    client.shutdown()
    for p in procs:
        try:
            p.wait(60)
        except subprocess.TimeoutExpired:
            p.kill()


def test_comet_sessions_and_duplicate_rejection():
    from moose_amd.runtime.choreography import ChoreographyClient

    port = _port()
    procs = _start(port)
    client = ChoreographyClient(f"127.0.0.1:{port}", timeout=240)
    try:
        comp_path = os.path.join(ROOT, "examples", "dot.moose")
        from moose_amd.cli.common import read_computation

        comp = read_computation(comp_path)
        outs, timings = client.run_computation("s1", comp, {}, IDS)
        np.testing.assert_allclose(outs["result"], [[1.0], [10.5]], atol=1e-5)
        assert set(timings) == set(IDS)
        with pytest.raises(RuntimeError, match="already exists"):
            client.launch_computation("s1", comp, {})
        client.abort_computation("s3")
        client.launch_computation("s3", comp, {})
        with pytest.raises(RuntimeError, match="aborted"):
            client.retrieve_results("s3", IDS, timeout=120)
        outs, _ = client.run_computation("s4", comp, {}, IDS)  # workers still serve
        np.testing.assert_allclose(outs["result"], [[1.0], [10.5]], atol=1e-5)
    finally:
        _stop(procs, client)


def test_filesystem_sessions(tmp_path):
    from moose_amd.runtime.choreography import ChoreographyClient

    for f in ("dot.moose", "dot.session"):
        shutil.copy(os.path.join(ROOT, "examples", f), tmp_path / f)
    port = _port()
    procs = _start(port, sessions_dir=str(tmp_path))
    client = ChoreographyClient(f"127.0.0.1:{port}", timeout=240)
    try:
        out = tmp_path / "dot.result.npy"
        deadline = time.time() + 180
        while not out.exists() and time.time() < deadline:
            time.sleep(0.2)
        assert out.exists()
        time.sleep(0.2)
        np.testing.assert_allclose(np.load(out), [[1.0], [10.5]], atol=1e-5)
    finally:
        _stop(procs, client)


def test_rudolph_no_listen_exits_after_existing_sessions(tmp_path):
    """``--no-listen``: run what is in the directory, then every worker exits by itself;
    ``--telemetry`` writes each worker's Chrome trace."""
    import json

    for f in ("dot.moose", "dot.session"):
        shutil.copy(os.path.join(ROOT, "examples", f), tmp_path / f)
    trace = str(tmp_path / "trace_{identity}.json")
    procs = _start(_port(), sessions_dir=str(tmp_path),
                   extra=("--no-listen", "--telemetry", trace))
    try:
        for p in procs:
            assert p.wait(180) == 0, p.stdout.read().decode()[-2000:]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    np.testing.assert_allclose(np.load(tmp_path / "dot.result.npy"), [[1.0], [10.5]],
                               atol=1e-5)
    for ident in IDS:
        with open(tmp_path / f"trace_{ident}.json") as f:
            evs = json.load(f)["traceEvents"]
        assert any(e["name"].startswith("op.") for e in evs)


def test_session_file_gpu_topology_and_replicas(tmp_path):
    """``[session] replicas`` / ``shard_args`` and per-role ``gpus``:
    parsed into a rank -> device map and run as 2 replicas x 3 parties (gloo here)."""
    import shutil

    import numpy as np

    from moose_amd.runtime.choreography import parse_session_file
    from moose_amd.runtime.choreography import run_session_file
    from moose_amd.runtime.choreography import session_device_map

    ex = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples")
    for f in ("dot_input.moose", "dot_replicas.session"):
        shutil.copy(os.path.join(ex, f), tmp_path / f)
    s = parse_session_file(str(tmp_path / "dot_replicas.session"))
    assert s["replicas"] == 2 and s["shard_args"] == ["x"]
    assert session_device_map(s) == [0, 1, 2, 3, 4, 5]
    x = np.arange(15, dtype=np.float64).reshape(5, 3) / 4
    outs, timings = run_session_file(str(tmp_path / "dot_replicas.session"), {"x": x},
                                     backend="gloo")
    np.testing.assert_allclose(outs["result"], x @ np.array([[2.0], [0.5], [-4.0]]), atol=1e-5)
    assert set(timings) == {"alice", "bob", "carole"}


def test_session_file_rejects_double_pinned_gpu(tmp_path):
    from moose_amd.runtime.choreography import parse_session_file
    from moose_amd.runtime.choreography import session_device_map

    (tmp_path / "c.moose").write_text("")
    (tmp_path / "s.session").write_text(
        '[computation]\npath = "c.moose"\n[[roles]]\nname = "a"\ngpu = 0\n'
        '[[roles]]\nname = "b"\ngpu = 0\n')
    import pytest

    with pytest.raises(ValueError):
        session_device_map(parse_session_file(str(tmp_path / "s.session")))
