"""cProfile of eager LR-inference evaluations on the GPU (host-side Python overhead)."""
import cProfile
import pstats
import sys

sys.path.insert(0, ".")


def main():
    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.runtime.local import LocalMooseRuntime

    tm = logistic_regression_tutorial(128)
    rt = LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", fixedpoint_ring=128)
    args = {"x": tm.x_test}
    for _ in range(5):
        rt.evaluate_computation(tm.computation, args)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        rt.evaluate_computation(tm.computation, args)
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
