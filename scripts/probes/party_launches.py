"""Native kernel launches per protocol step of ONE party of the tutorial LR inference (the
in-process parties on the CPU: the same per-party code path as on the GPU), plus the torch
copies / concatenations a GPU evaluation would launch.  Prints a markdown tree like
scripts/lr_rounds.py, with launches instead of rounds."""
import argparse
import collections
import functools
import inspect
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--party", default="alice")
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    import numpy as np
    import torch

    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.ops import native as nat
    from moose_amd.protocols import fixedpoint as FP
    from moose_amd.protocols import replicated as REP
    from moose_amd.runtime.local import LocalMooseRuntime

    tls = threading.local()
    acc = collections.defaultdict(collections.Counter)
    rounds = collections.Counter()
    order = []

    def stack():
        s = getattr(tls, "s", None)
        if s is None:
            s = tls.s = []
        return s

    def wrap(mod, name, fn):
        @functools.wraps(fn)
        def w(*args, **kw):
            s = stack()
            if len(s) >= a.depth:
                return fn(*args, **kw)
            s.append(f"{mod}.{name}")
            key = tuple(s)
            sess = args[0] if args else None
            st = getattr(sess, "stats", None)
            mine = threading.current_thread().name == f"moose-party-{a.party}"
            r0 = st.rounds if st is not None else 0
            try:
                return fn(*args, **kw)
            finally:
                if st is not None and mine:
                    if key not in acc:
                        order.append(key)
                        acc[key]  # noqa: B018 - create the row
                    rounds[key] += st.rounds - r0
                s.pop()
        return w

    for mod, m in (("fp", FP), ("rep", REP)):
        for name, fn in list(vars(m).items()):
            if inspect.isfunction(fn) and fn.__module__ == m.__name__:
                setattr(m, name, wrap(mod, name, fn))

    def note(what):
        if threading.current_thread().name != f"moose-party-{a.party}":
            return
        key = tuple(stack()) or ("(interpreter)",)
        if key not in acc:
            order.append(key)
        acc[key][what] += 1

    lib = nat.lib()

    class Proxy:
        def __getattr__(self, name):
            f = getattr(lib, name)
            if not name.startswith("mx_") or name in ("mx_version",):
                return f

            def call(*args):
                note(name)
                return f(*args)
            return call

    proxy = Proxy()
    nat.lib = lambda: proxy
    for tname in ("cat", "stack"):
        orig = getattr(torch, tname)

        def mk(orig, tname):
            def f(*x, **k):
                note(f"torch.{tname}")
                return orig(*x, **k)
            return f
        setattr(torch, tname, mk(orig, tname))
    orig_copy = torch.Tensor.copy_

    def copy_(self, *x, **k):
        note("torch.copy_")
        return orig_copy(self, *x, **k)
    torch.Tensor.copy_ = copy_

    ids = ["alice", "bob", "carole"]
    tm = logistic_regression_tutorial(a.batch)
    rt = LocalMooseRuntime(ids, device_map={i: "cpu" for i in ids}, seed=1)
    r = list(rt.evaluate_computation(tm.computation, {"x": tm.x_test}).values())[0]
    err = float(np.abs(np.asarray(r) - tm.proba).max())
    total = sum(sum(c.values()) for c in acc.values())
    print(f"# launches of party {a.party} per LR evaluation: {total} (err {err:.1e}); "
          f"rounds {rt.last_stats.rounds}\n")
    print("| step | rounds (incl.) | launches | by kernel |\n|---|---|---|---|")
    for key in order:
        c = acc[key]
        ind = "&nbsp;" * 4 * (len(key) - 1)
        top = ", ".join(f"{k.replace('mx_', '')} {v}" for k, v in c.most_common())
        print(f"| {ind}{key[-1]} | {rounds[key]} | {sum(c.values())} | {top} |")


if __name__ == "__main__":
    main()
