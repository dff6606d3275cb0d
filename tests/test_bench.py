"""bench.py contract on CPU (gloo): one JSON line from rank 0 with the driver's fields, for
the default stacked data-parallel layout and the party-per-GPU (SPMD) layout."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
          "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(n, *extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py",
           "--gpus", str(n), "--steps", "2", "--warmup", "1", "--size", "64", *extra]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    return json.loads(lines[0])


@pytest.mark.parametrize("n,layout", [(2, "stacked"), (3, "spmd")])
def test_bench_json_line(n, layout):
    d = _run(n, "--layout", layout)
    assert FIELDS <= set(d)
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1
    assert d["value"] > 0 and d["higher_is_better"] is True
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(d["config"])


def _run_self(n, *extra):
    """No launcher: bench.py --gpus N spawns its N ranks itself."""
    cmd = [sys.executable, "bench.py", "--gpus", str(n), "--steps", "2", "--warmup", "1",
           "--size", "48", "--check", *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    return json.loads(lines[0])


@pytest.mark.parametrize("n,layout,sessions", [(2, "auto", 2), (3, "spmd", 1), (4, "cyclic", 4)])
def test_bench_self_launch(n, layout, sessions):
    d = _run_self(n, "--layout", layout)
    assert FIELDS <= set(d)
    assert d["n_gpus"] == n and d["world_size"] == n and d["sessions"] == sessions
    assert d["layout"] == ("cyclic" if layout == "auto" else layout)
    assert len(d["per_rank_ms_per_step"]) == n
    assert d["ms_per_step"] == pytest.approx(max(d["per_rank_ms_per_step"]))
    assert d["check"] and all(c["max_abs_err"] < 1e-4 for c in d["check"])
    if sessions > 1:  # rank 0 (the client) collected every session's revealed output
        assert d["gather"] == "root" and d["check"][0]["gathered_max_abs_err"] < 1e-4
