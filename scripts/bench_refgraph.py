"""Execute the reference lowered benchmark graph (rep_computation.moose) with the graph
executor: python scripts/bench_refgraph.py [cpu|cuda] [path]."""
import time, sys
import numpy as np, torch
from moose_amd.ir.computation import Computation
from moose_amd.compiler import passes
from moose_amd.runtime.graph_executor import GraphExecutor
dev = sys.argv[1] if len(sys.argv) > 1 else "cpu"
src = open(sys.argv[2] if len(sys.argv) > 2 else '/root/reference/moose/benches/rep_computation.moose').read()
t = time.time(); c = Computation.from_textual(src, parallel=False); print("parse", time.time() - t)
t = time.time(); c = passes.compile(c, ["networking", "toposort"]); print("networking+toposort", time.time() - t, len(c.operations))
storage = {}
ex = GraphExecutor(dev, storage)
for i in range(3):
    t = time.time(); ex.run(c, {})
    if dev != "cpu": torch.cuda.synchronize()
    print("run", i, time.time() - t)
print(storage)
