"""Count torch tensor-function calls by moose_amd call site during one private LR inference
(TorchFunctionMode; works on the GPU): which Python sites produce the ATen copy kernels."""
import collections
import os
import sys
import traceback

import numpy as np
import torch
from torch.overrides import TorchFunctionMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

WATCH = {"roll", "stack", "clone", "contiguous", "cat", "zeros", "zeros_like", "empty_like",
         "copy_", "to", "__setitem__", "expand", "where", "full", "__and__", "__xor__",
         "__lshift__", "__rshift__", "__or__", "add", "sub", "mul", "__add__", "__sub__",
         "flip", "narrow", "index_select", "gather", "scatter", "fill_", "new_zeros"}


class Count(TorchFunctionMode):
    def __init__(self):
        super().__init__()
        self.where = collections.Counter()

    def __torch_function__(self, func, types, args=(), kwargs=None):
        name = getattr(func, "__name__", str(func))
        if name == "contiguous" and args and args[0].is_contiguous():
            name = None  # no copy
        if name in WATCH:
            st = [f for f in traceback.extract_stack(limit=30) if "moose_amd" in f.filename]
            if st:
                # the kernel's site plus the protocol frames that asked for it
                outer = [f for f in st[:-1] if "protocols/" in f.filename][-2:]
                self.where[(name,) + tuple(
                    f.filename.split("moose_amd/")[-1] + ":" + str(f.lineno) + " " + f.name
                    for f in outer + [st[-1]])] += 1
        return func(*args, **(kwargs or {}))


def main():
    from sklearn.datasets import make_classification
    from sklearn.linear_model import LogisticRegression

    from moose_amd.models import predictors
    from moose_amd.runtime.local import LocalMooseRuntime

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    X, y = make_classification(n_samples=1000, n_features=10, n_classes=2, random_state=5)
    lg = LogisticRegression().fit(X[:800], y[:800])
    model = predictors.LinearClassifier(np.stack([-lg.coef_[0], lg.coef_[0]]),
                                        np.array([-lg.intercept_[0], lg.intercept_[0]]),
                                        predictors.PostTransform.SIGMOID)
    comp = model.predictor_factory(predictors.DEFAULT_FIXED_DTYPE)
    rt = LocalMooseRuntime(["alice", "bob", "carole"], device=dev, use_graphs=False)
    for _ in range(2):
        rt.evaluate_computation(comp, {"x": X[800:]})
    c = Count()
    with c:
        rt.evaluate_computation(comp, {"x": X[800:]})
    for k, v in c.where.most_common(60):
        print(v, k)


if __name__ == "__main__":
    main()
