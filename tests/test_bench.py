"""bench.py contract on CPU (gloo): one JSON line from rank 0 with the driver's fields, for
the default stacked data-parallel layout and the party-per-GPU (SPMD) layout."""
import json
import os
import socket
import subprocess
import sys
import time

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
           "--gpus", str(n), "--steps", "2", "--warmup", "1", "--size", "64", "--lr-runs", "0",
           *extra]
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
           "--size", "48", "--lr-runs", "0", *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    return json.loads(lines[0])


@pytest.mark.parametrize("n,layout,sessions", [(2, "auto", 2), (3, "spmd", 1), (4, "cyclic", 4),
                                               (3, "auto", 3)])
def test_bench_self_launch(n, layout, sessions):
    d = _run_self(n, "--layout", layout)
    assert FIELDS <= set(d)
    assert d["n_gpus"] == n and d["world_size"] == n and d["sessions"] == sessions
    assert d["layout"] == ({2: "stacked"}.get(n, "cyclic") if layout == "auto" else layout)
    assert len(d["per_rank_ms_per_step"]) == n
    assert d["ms_per_step"] == pytest.approx(max(d["per_rank_ms_per_step"]))
    # every output owner checked its last output (and rank 0 the collected outputs)
    assert d["check"]["ok"] and d["check"]["max_abs_err"] < 1e-4
    assert d["check"]["ranks"] == (1 if layout == "spmd" else n)
    assert d["preflight"]["ok"]
    assert len(d["p2p_bytes_per_step"]) == n
    if sessions > 1:  # rank 0 (the client) collected every session's revealed output
        assert d["gather"] == "root"
    if d["layout"] == "cyclic":  # every reshare crossed ranks
        assert min(d["p2p_bytes_per_step"]) > 0 and d["step_streams"] == 2
        # after the headline: point-to-point GB/s of the layout's exchange pattern
        assert all(v > 0 for v in d["link_probe"]["gbs_per_rank_and_direction"].values())
        # small-message latency of one grouped exchange per distance (8 B, 4 KB, 64 KB)
        lat = d["link_probe"]["exchange_latency_us_p50"]
        assert len(lat) == 3 * (len(d["link_probe"]["gbs_per_rank_and_direction"]) - 1)
        assert all(v > 0 for v in lat.values())


def test_bench_lr_inference_in_line():
    """The second half of the headline metric: LR-inference p50 in the same JSON line
    (one GPU eager/graphs, and with >= 3 ranks one party per rank)."""
    cmd = [sys.executable, "bench.py", "--gpus", "3", "--steps", "1", "--warmup", "1",
           "--size", "32", "--lr-runs", "2"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    p50 = d["lr_inference_p50_ms"]
    assert {"eager", "graphs", "spmd"} <= set(p50) and all(v > 0 for v in p50.values())
    lr = d["lr_inference"]
    assert lr["one_gpu"]["eager"]["max_abs_err_vs_sklearn"] < 1e-3
    assert lr["spmd_one_party_per_gpu"]["eager"]["max_abs_err_vs_sklearn"] < 1e-3
    assert d["lr_inference_rounds"] > 0
    # BASELINE configs 2 and 3 with one party per rank (the reference's dotprod.moose: 32)
    sp = d["spmd_three_gpus"]
    assert sp["config2_dotprod_moose"]["output"] == pytest.approx(32.0, abs=1e-6)
    assert sp["config2_dotprod_moose"]["p50_ms"] > 0
    assert sp["config3_ringdot_3gpu"]["ms_per_step"] > 0


def _run_env(n, env_extra, *extra, timeout=300):
    cmd = [sys.executable, "bench.py", "--gpus", str(n), "--steps", "2", "--warmup", "1",
           "--size", "32", "--lr-runs", "0", *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    t0 = time.monotonic()
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                         env=env)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (out.stdout[-2000:], out.stderr[-3000:])
    return out.returncode, json.loads(lines[0]), time.monotonic() - t0


@pytest.mark.parametrize("phase,rank", [("timed", 2), ("preflight", 1)])
def test_bench_stalled_rank_fails_loudly(phase, rank):
    """A rank that hangs in every attempt of the fallback ladder: bench.py --gpus 3 exits
    non-zero inside its deadline with an error line naming the stalled rank and listing
    every attempt."""
    rc, d, secs = _run_env(3, {"MOOSEX_BENCH_STALL": f"{rank}:{phase}:*"}, "--deadline", "90")
    assert rc != 0 and secs < 90 + 45
    assert d["value"] is None and "error" in d
    assert d["stalled_ranks"] == [rank]
    assert [a["outcome"] for a in d["attempts"]] == ["failed"] * 3
    assert all(a["phase"] == phase for a in d["attempts"])
    assert [(a["layout"], a["streams"]) for a in d["attempts"]] == [
        ("cyclic", 2), ("cyclic", 1), ("stacked", 1)]


def test_bench_fallback_ladder_recovers_a_stalled_attempt():
    """A rank that hangs in the warmup of the first attempt (cyclic, two step streams): the
    supervisors kill that attempt on every rank and the next rung (one step stream)
    measures the headline, well inside the deadline; the line carries both attempts."""
    rc, d, secs = _run_env(3, {"MOOSEX_BENCH_STALL": "1:warmup"}, "--step-streams", "2",
                           "--deadline", "150")
    assert rc == 0 and secs < 150
    assert d["value"] > 0 and d["check"]["ok"] and d["fallback"] is True
    a0, a1 = d["attempts"]
    assert (a0["layout"], a0["streams"], a0["outcome"], a0["phase"]) == (
        "cyclic", 2, "failed", "warmup")
    assert a0["stalled_ranks"] == [1]
    assert (a1["layout"], a1["streams"], a1["outcome"]) == ("cyclic", 1, "ok")
    assert d["step_streams"] == 1
    # per-phase wall times of the attempt that measured
    assert {"init", "rendezvous", "preflight", "warmup", "timed"} <= set(d["phase_s"])


def _benchwatch():
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "bw", os.path.join(ROOT, "moose_amd", "utils", "benchwatch.py"))
    bw = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bw)
    return bw


def test_phase_budgets_are_clipped_to_the_deadline(tmp_path):
    """Budgets come out of one deadline: a phase's watchdog budget is its cap clipped to
    the time left (before the headline: to the attempt's headline deadline), and an extra
    whose expected need no longer fits is reported as not fitting (then skipped)."""
    bw = _benchwatch()
    now = time.time()
    clock = bw.Clock(now + 40, now + 20, 1.0)
    p = bw.Progress(0, 1, clock, lambda: {}, directory=str(tmp_path))
    p.phase("warmup")  # cap 120 s, clipped to the headline deadline (20 s - margin)
    assert p.deadline - time.monotonic() < 20
    p.headline_done({"value": 1.0})
    p.phase("check")  # after the headline: clipped to the run's deadline instead
    assert 20 < p.deadline - time.monotonic() < 40
    assert p.extra_fits("check") and not p.extra_fits("spmd_configs")  # need 10 s vs 45 s
    p.skip("spmd_configs")
    line = p.final_line()
    assert line["skipped"] == ["spmd_configs"] and {"init", "warmup"} <= set(line["phase_s"])
    p.disarm()


def test_supervisor_kills_a_hung_rank_group(tmp_path):
    """The self-launch parent's wall-clock limit: a child group that never finishes is
    killed and an error line is printed from the phase files."""
    bw = _benchwatch()
    (tmp_path / "rank0.json").write_text(json.dumps({"phase": "timed", "seq": 4, "step": 3}))
    (tmp_path / "rank1.json").write_text(json.dumps({"phase": "timed", "seq": 4, "step": 0}))
    import contextlib
    import io

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = bw.supervise([sys.executable, "-c", "import time; time.sleep(600)"], dict(os.environ),
                          2, 2.0, {"metric": "m"}, str(tmp_path))
    d = json.loads(buf.getvalue().strip().splitlines()[-1])
    assert rc == 3 and d["stalled_ranks"] == [1] and "error" in d


@pytest.mark.parametrize("phase,rank,headline", [("lr_spmd", 1, True), ("warmup", 2, False)])
def test_bench_rank_exception_ends_the_run_promptly(phase, rank, headline):
    """A rank that raises ends its attempt on every rank at once (its peers' watchdogs read
    its failure record instead of waiting out their phase budget).  After the headline was
    measured (an optional extra failed) the line keeps the measurement and notes the error;
    before it, the next rung of the ladder measures instead."""
    cmd = [sys.executable, "bench.py", "--gpus", "3", "--steps", "1", "--warmup", "1",
           "--size", "32", "--lr-runs", "2", "--deadline", "200"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MOOSEX_BENCH_FAIL"] = f"{rank}:{phase}"
    t0 = time.monotonic()
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400, env=env)
    assert time.monotonic() - t0 < 120  # far inside the 200 s phase budget
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert out.returncode == 0, out.stderr[-2000:]
    assert d["value"] > 0 and d["check"]["ok"]
    if headline:
        assert d["errors"][0]["phase"] == phase
        assert len(d["attempts"]) == 1
    else:
        a0 = d["attempts"][0]
        assert a0["outcome"] == "failed" and f"rank {rank}" in a0["error"]
        assert d["attempts"][1]["outcome"] == "ok"


def test_bench_config5_two_replicas_on_six_ranks():
    """BASELINE config 5: two data-parallel replicas of the 3-party session on six ranks,
    RingDot per replica with every reshare cross-rank, both revealed outputs all-gathered
    between the replicas' clients and checked."""
    d = _run_self(6, "--layout", "cyclic")
    c5 = d["config5_dp2_replicas"]
    assert c5["replicas"] == 2 and c5["dots_per_step"] == 2 and c5["ms_per_step"] > 0
    assert c5["gathered_max_abs_err"] < 1e-3
    assert d["spmd_three_gpus"]["config2_dotprod_moose"]["output"] == pytest.approx(32.0)



def _gpus():
    try:
        import torch

        return torch.cuda.device_count()  # counting does not initialise the GPU
    except Exception:  # noqa: BLE001
        return 0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [3, 6])
def test_bench_rccl_multi_gpu(n):
    """The driver's multi-GPU bench path on real GPUs (one rank per GPU, RCCL): cyclic
    headline with its output check, LR inference one party per GPU, configs 2/3 (and 5 on
    six GPUs).  Gated on the device count, as SURVEY section 4 asks."""
    if _gpus() < n:
        pytest.skip(f"needs {n} GPUs")
    cmd = [sys.executable, "bench.py", "--gpus", str(n), "--steps", "2", "--warmup", "1",
           "--size", "1024", "--lr-runs", "3", "--deadline", "400"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MOOSEX_SHARED_GPU")}
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert "errors" not in d, d.get("errors")
    assert d["layout"] == "cyclic" and d["check"]["ok"] and d["preflight"]["ok"]
    assert min(d["p2p_bytes_per_step"]) > 0
    assert d["spmd_three_gpus"]["config2_dotprod_moose"]["output"] == pytest.approx(32.0)
    sp = d["lr_inference"]["spmd_one_party_per_gpu"]
    assert sp["eager"]["max_abs_err_vs_sklearn"] < 1e-3
    assert sp["tape"]["replayed"] and sp["tape"]["max_abs_err_vs_sklearn"] < 1e-3
    if n >= 6:
        assert d["config5_dp2_replicas"]["gathered_max_abs_err"] < 1e-2
