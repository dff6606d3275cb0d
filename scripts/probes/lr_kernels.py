"""LR inference (tutorial model) with hipGraph replay, for a kernel trace: 30 replays."""
import sys

sys.path.insert(0, ".")


def main():
    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.runtime.local import LocalMooseRuntime

    tm = logistic_regression_tutorial(128)
    rt = LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", fixedpoint_ring=128,
                           use_graphs=True)
    for _ in range(33):
        rt.evaluate_computation(tm.computation, {"x": tm.x_test})


if __name__ == "__main__":
    main()
