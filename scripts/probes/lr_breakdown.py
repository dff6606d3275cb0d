"""Where the host time of one hipGraph-replayed LR inference goes (runtime/graphs.py):
wall time of evaluate_computation and, inside GraphPlan.run, the host time of each phase
(argument upload, key refresh, graph launches, decode incl. the D2H read-back)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")


def main():
    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.runtime import graphs
    from moose_amd.runtime.local import LocalMooseRuntime

    tm = logistic_regression_tutorial(128)
    rt = LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", fixedpoint_ring=128,
                           use_graphs=True)
    args = {"x": tm.x_test}
    phases = {"upload": [], "refresh": [], "replay": [], "decode": []}
    orig_run = graphs.GraphPlan.run

    def run(self, arguments):
        t0 = time.perf_counter()
        for k, v in arguments.items():
            t = self.static.get(k)
            if hasattr(t, "copy_"):
                a = np.asarray(v)
                import torch
                t.copy_(torch.from_numpy(np.ascontiguousarray(a).reshape(t.shape)))
        t1 = time.perf_counter()
        self.keys.refresh(self.keys.n)
        t2 = time.perf_counter()
        for g in self.graphs:
            g.replay()
        t3 = time.perf_counter()
        self.replays += 1
        out = self._decode(self.interp, self.outs)
        t4 = time.perf_counter()
        for k, a, b in (("upload", t0, t1), ("refresh", t1, t2), ("replay", t2, t3),
                        ("decode", t3, t4)):
            phases[k].append((b - a) * 1e3)
        return out

    graphs.GraphPlan.run = run
    walls = []
    for i in range(80):
        t0 = time.perf_counter()
        rt.evaluate_computation(tm.computation, args)
        walls.append((time.perf_counter() - t0) * 1e3)
    graphs.GraphPlan.run = orig_run
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(json.dumps({"wall_p50_ms": med(walls[20:]),
                      **{k: round(med(v[20:]), 4) for k, v in phases.items()},
                      "graphs": len(next(iter(rt._graphs.plans.values())).graphs)
                      if getattr(rt, "_graphs", None) else None}))


if __name__ == "__main__":
    main()
