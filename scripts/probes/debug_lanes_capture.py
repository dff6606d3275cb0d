"""Capture the independent-branches computation with dataflow lanes (debug helper)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import moose_amd as pm
    from moose_amd.runtime import graphs
    from tests.test_lanes import _wide_comp

    branches = int(os.environ.get("BR", "2"))
    lanes = int(os.environ.get("LANES", "2"))
    if os.environ.get("SEG"):
        graphs.SEGMENT_OPS = int(os.environ["SEG"])
    f, x, ref = _wide_comp(branches, int(os.environ.get("ROWS", "16")))
    for ln in [int(v) for v in os.environ.get("SEQ", str(lanes)).split(",")]:
        rt = pm.LocalMooseRuntime(["alice", "bob", "carole"], device="cuda", use_graphs=True,
                                  lanes=ln)
        for i in range(3):
            r = rt.evaluate_computation(f, {"x": x})
            print("lanes", ln, "eval", i, "plans", len(rt._graphs.plans), flush=True)


if __name__ == "__main__":
    main()
