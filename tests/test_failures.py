"""Failure detection and recovery: a dropped message trips the per-session
deadline instead of hanging, a fresh session then succeeds; lowered graphs enforce
exactly-once rendezvous; telemetry spans export as a Chrome trace."""
import json
import os

import numpy as np
import pytest

import moose_amd as pm
from moose_amd.compiler import passes
from moose_amd.ir.computation import Computation
from moose_amd.runtime.distributed import DistributedMooseRuntime
from moose_amd.runtime.distributed import DistributedRuntimeError
from moose_amd.runtime.graph_executor import GraphExecutionError
from moose_amd.runtime.graph_executor import GraphExecutor

IDS = ["alice", "bob", "carole"]


def _comp():
    alice, bob, carole = (pm.host_placement(n) for n in IDS)
    rep = pm.replicated_placement("rep", players=[alice, bob, carole])

    @pm.computation
    def f(x: pm.Argument(alice, vtype=pm.TensorType(pm.float64))):
        with alice:
            xf = pm.cast(x, dtype=pm.fixed(14, 23))
        with rep:
            y = pm.mul(xf, xf)
        with bob:
            return pm.cast(y, dtype=pm.float64)

    return f


def test_dropped_message_hits_deadline_then_fresh_session_succeeds():
    x = np.array([1.5, -2.0])
    rt = DistributedMooseRuntime(IDS, backend="gloo", timeout=120, session_timeout=5,
                                 worker_env={"MOOSEX_FAULT": "drop:3@0"})
    with pytest.raises(DistributedRuntimeError):
        rt.evaluate_computation(_comp(), {"x": x})
    rt.worker_env = {}
    out = rt.evaluate_computation(_comp(), {"x": x})
    np.testing.assert_allclose(list(out.values())[0], x * x, atol=1e-5)


def test_lowered_graph_rejects_duplicate_sends():
    src = """
a = Constant{value = HostFloat64Tensor([1.0])}: () -> HostFloat64Tensor () @Host(alice)
s1 = Send{rendezvous_key = 01, receiver = "bob"}: (HostFloat64Tensor) -> HostUnit (a) @Host(alice)
s2 = Send{rendezvous_key = 01, receiver = "bob"}: (HostFloat64Tensor) -> HostUnit (a) @Host(alice)
r = Receive{rendezvous_key = 01, sender = "alice"}: () -> HostFloat64Tensor () @Host(bob)
o = Output{tag = "o"}: (HostFloat64Tensor) -> HostFloat64Tensor (r) @Host(bob)
"""
    with pytest.raises(GraphExecutionError, match="duplicate send"):
        GraphExecutor("cpu").run(Computation.from_textual(src), {})


def test_chrome_trace_and_session_stats(tmp_path):
    from moose_amd.runtime.local import LocalMooseRuntime
    from moose_amd.utils import telemetry

    path = tmp_path / "trace.json"
    old = telemetry._TRACE_PATH
    telemetry._TRACE_PATH = str(path)
    try:
        rt = LocalMooseRuntime(IDS, device="cpu")
        rt.evaluate_computation(_comp(), {"x": np.array([1.0, 2.0])})
        telemetry.dump_trace()
    finally:
        telemetry._TRACE_PATH = old
    evs = json.load(open(path))["traceEvents"]
    names = {e["name"] for e in evs}
    # the fixed-point product runs as the per-party folded tail (rep.mul_trunc_party)
    assert "rep.mul_trunc_party" in names and "rep.reveal" in names and "op.Mul" in names
    stats = rt.last_stats.as_dict()
    assert stats["rounds"] >= 2 and any(v > 0 for v in stats["bytes"].values())
    assert set(rt.last_timings) == set(IDS)


def test_lowered_plan_is_deterministic_textual():
    comp = passes.compile(Computation.from_textual(
        'c = Constant{value = HostFloat64Tensor([1.0, 2.0])}: () -> Tensor<Float64> () @Host(a)\n'
        'f = Cast: (Tensor<Float64>) -> Tensor<Fixed128(14, 23)> (c) @Host(a)\n'
        'm = Mul: (Tensor<Fixed128(14, 23)>, Tensor<Fixed128(14, 23)>) -> Tensor<Fixed128(14, 23)> (f, f) @Replicated(a, b, c)\n'
        'o = Output{tag = "o"}: (Tensor<Fixed128(14, 23)>) -> Tensor<Fixed128(14, 23)> (m) @Host(b)\n'))
    again = passes.compile(Computation.from_textual(
        'c = Constant{value = HostFloat64Tensor([1.0, 2.0])}: () -> Tensor<Float64> () @Host(a)\n'
        'f = Cast: (Tensor<Float64>) -> Tensor<Fixed128(14, 23)> (c) @Host(a)\n'
        'm = Mul: (Tensor<Fixed128(14, 23)>, Tensor<Fixed128(14, 23)>) -> Tensor<Fixed128(14, 23)> (f, f) @Replicated(a, b, c)\n'
        'o = Output{tag = "o"}: (Tensor<Fixed128(14, 23)>) -> Tensor<Fixed128(14, 23)> (m) @Host(b)\n'))
    assert comp.digest() == again.digest()
    assert os.environ.get("MOOSEX_FAULT") is None


def test_error_model_variants():
    """Reference error.rs:7-61: 17 variants; subsystem errors map onto them."""
    from moose_amd import errors
    from moose_amd.compiler.passes import CompilationError
    from moose_amd.ir.textual import ParseError
    from moose_amd.ops.native import NativeError
    from moose_amd.parallel.transport import TransportError
    from moose_amd.runtime.graph_executor import GraphExecutionError
    from moose_amd.runtime.interpreter import MooseRuntimeError

    assert len(errors.VARIANTS) == 17
    assert all(issubclass(v, errors.MooseError) for v in errors.VARIANTS)
    assert issubclass(CompilationError, errors.Compilation)
    assert issubclass(ParseError, errors.MalformedComputation) and issubclass(ParseError, ValueError)
    assert issubclass(NativeError, errors.KernelError)
    assert issubclass(TransportError, errors.Networking)
    assert issubclass(GraphExecutionError, errors.KernelError)
    assert issubclass(MooseRuntimeError, errors.KernelError)


def test_gemm_workspace_failure_names_the_size(monkeypatch):
    """a GEMM whose device workspace cannot be allocated (code -4)
    raises an error that names the size it tried and what is already held."""
    import pytest

    from moose_amd.ops import native

    monkeypatch.setattr(native, "_ws_failed_bytes", lambda: 8 << 30)
    monkeypatch.setattr(native, "_ws_held_bytes", lambda: 24 << 30)
    with pytest.raises(native.NativeError) as e:
        native.check(-4, "ring gemm")
    msg = str(e.value)
    assert "8.00 GiB" in msg and "8589934592 bytes" in msg and "24.00 GiB" in msg
    assert "docs/API.md" in msg
