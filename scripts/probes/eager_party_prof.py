"""Where an EAGER per-party evaluation's host time goes (one small dot, parties as threads
on one GPU): cProfile of party alice's interpreter thread and of the calling thread."""
import cProfile
import io
import os
import pstats
import sys
import threading
import time

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "benchmarks"))


def main():
    import numpy as np

    from dot_product import build
    from moose_amd.runtime.interpreter import Interpreter
    from moose_amd.runtime.local import LocalMooseRuntime, to_native

    k = int(os.environ.get("EAGER_K", "1"))
    native = to_native(build("seq", k))
    args = {"x_arg": np.ones((1, 1)), "y_arg": np.identity(1)}
    ids = ["alice", "bob", "carole"]
    rt = LocalMooseRuntime(ids, device_map={i: "cuda:0" for i in ids}, use_graphs=False,
                           timeout=60)
    for _ in range(3):
        rt.evaluate_computation(native, args)
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        rt.evaluate_computation(native, args)
        ts.append((time.perf_counter() - t0) * 1e3)
    print("eager per-party dot p50 ms", sorted(ts)[10], dict(rt.last_timings), flush=True)
    prof = []
    orun = Interpreter.run

    def prun(self, *a, **k):
        if threading.current_thread().name.endswith("alice"):
            pr = cProfile.Profile()
            pr.enable()
            try:
                return orun(self, *a, **k)
            finally:
                pr.disable()
                prof.append(pr)
        return orun(self, *a, **k)

    Interpreter.run = prun
    main_pr = cProfile.Profile()
    main_pr.enable()
    for _ in range(10):
        rt.evaluate_computation(native, args)
    main_pr.disable()
    for name, ps in (("alice thread", prof), ("caller", [main_pr])):
        st = pstats.Stats(ps[0], stream=io.StringIO())
        for p in ps[1:]:
            st.add(p)
        s = io.StringIO()
        st.stream = s
        st.sort_stats(os.environ.get("EAGER_SORT", "tottime")).print_stats(
            int(os.environ.get("EAGER_TOP", "16")))
        print(f"== {name}\n" + s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
