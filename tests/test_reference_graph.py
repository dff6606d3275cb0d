"""Runs the reference's own lowered benchmark computation
(``moose/benches/rep_computation.moose``: 19,045 host operations -- RSS sharing, bit
decomposition, Kogge-Stone adders, the exp protocol on a replicated placement --
produced by the reference's compiler) through our networking pass and graph executor.
The graph computes exp(2.0) and saves it on alice.  The file is read from the
reference checkout when present (it is not copied into this repository)."""
import os

import numpy as np
import pytest

from moose_amd.compiler import passes
from moose_amd.ir.computation import Computation
from moose_amd.runtime.graph_executor import GraphExecutor

REF = "/root/reference/moose/benches/rep_computation.moose"


@pytest.mark.skipif(not os.path.exists(REF), reason="reference checkout not available")
def test_reference_benchmark_graph_computes_exp2():
    with open(REF) as f:
        comp = Computation.from_textual(f.read(), parallel=False)
    assert len(comp.operations) == 19045
    comp = passes.compile(comp, ["networking", "toposort", "wellformed"])
    storage = {}
    GraphExecutor("cpu", storage).run(comp, {})
    np.testing.assert_allclose(np.asarray(storage["alice"]["y_uri"]), [np.exp(2.0)], rtol=1e-5)
