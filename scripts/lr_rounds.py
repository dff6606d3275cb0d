"""Message rounds of the tutorial LR inference, per protocol step.

Runs the ml-inference-with-onnx tutorial model (fixed(24,40), Z_2^128) once on a CPU
session -- by default the per-party protocol of the SPMD and multi-GPU layouts (a
one-process cyclic session: its ``stats.rounds`` is what an SPMD evaluation records) --
with every public function of
``protocols/fixedpoint.py`` and ``protocols/replicated.py`` wrapped, and prints the rounds
each logical operation and each protocol step under it took (inclusive), as a markdown
tree.  ``--json`` writes the same data.
"""
import argparse
import functools
import inspect
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--json", default=None)
    ap.add_argument("--layout", default="party", choices=["party", "stacked"],
                    help="party: the per-party protocol (a one-process cyclic session, as "
                         "SPMD and the multi-GPU layouts run it); stacked: the simulation")
    a = ap.parse_args()

    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.protocols import fixedpoint as FP
    from moose_amd.protocols import replicated as REP
    from moose_amd.runtime import interpreter as I
    from moose_amd.runtime.local import to_native
    from moose_amd.runtime.session import StackedSession

    stack, acc, order = [], {}, []
    cur = {"sess": None}

    def rounds():
        return cur["sess"].stats.rounds

    def wrap(mod, name, fn):
        @functools.wraps(fn)
        def w(*args, **kw):
            if cur["sess"] is None or len(stack) >= a.depth:
                return fn(*args, **kw)
            stack.append(f"{mod}.{name}")
            key = tuple(stack)
            if key not in acc:
                order.append(key)
                acc[key] = [0, 0]
            r0 = rounds()
            try:
                return fn(*args, **kw)
            finally:
                acc[key][0] += rounds() - r0
                acc[key][1] += 1
                stack.pop()
        return w

    for mod, m in (("fp", FP), ("rep", REP)):
        for name, fn in list(vars(m).items()):
            if inspect.isfunction(fn) and fn.__module__ == m.__name__ and not name.startswith("__"):
                setattr(m, name, wrap(mod, name, fn))
    run_op = I.Interpreter._run_op

    def run_op_w(self, op, *args):
        stack.append(f"op {op.kind} ({op.name})")
        key = tuple(stack)
        if key not in acc:
            order.append(key)
            acc[key] = [0, 0]
        r0 = rounds()
        try:
            return run_op(self, op, *args)
        finally:
            acc[key][0] += rounds() - r0
            acc[key][1] += 1
            stack.pop()

    I.Interpreter._run_op = run_op_w
    tm = logistic_regression_tutorial(128)
    comp = to_native(tm.computation, 128)
    if a.layout == "stacked":
        sess = StackedSession("cpu", seed=1)
    else:
        from moose_amd.parallel.cyclic import CyclicSession
        from moose_amd.parallel.cyclic import RingComm

        sess = CyclicSession(RingComm(0, 1, "cpu"), {"alice": 0, "bob": 0, "carole": 0},
                             "cpu", seed=1)
    cur["sess"] = sess
    I.Interpreter(sess, {}, 128).run(comp, {"x": tm.x_test})
    total = sess.stats.rounds
    rows = [(k, v[0], v[1]) for k, v in ((k, acc[k]) for k in order) if v[0] > 0]
    print(f"# Message rounds of one tutorial LR inference ({a.layout}): {total}\n")
    print("| step | rounds (inclusive) | calls |")
    print("|---|---|---|")
    for k, r, c in rows:
        print(f"| {'&nbsp;&nbsp;' * 2 * (len(k) - 1)}{k[-1]} | {r} | {c} |")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"total": total, "rows": [[list(k), r, c] for k, r, c in rows]}, f)


if __name__ == "__main__":
    main()
