"""``from_onnx``: infer the predictor type of an ONNX model.

Parity: reference ``pymoose/pymoose/predictors/onnx_convert.py:8-92``: PyTorch and
tf2onnx exports are neural networks; otherwise the single recognised ML operator
(LinearRegressor / LinearClassifier / TreeEnsembleRegressor / TreeEnsembleClassifier)
decides, and graphs with several weight matrices are sklearn MLPs (classifiers have a
``ZipMap`` node).
"""
from __future__ import annotations

from moose_amd.models.predictors import linear
from moose_amd.models.predictors import neural
from moose_amd.models.predictors import trees
from moose_amd.models.predictors.base import load_onnx

_SUPPORTED = {
    "LinearRegressor": linear.LinearRegressor,
    "LinearClassifier": linear.LinearClassifier,
    "TreeEnsembleRegressor": trees.TreeEnsembleRegressor,
    "TreeEnsembleClassifier": trees.TreeEnsembleClassifier,
}


def from_onnx(model):
    model = load_onnx(model)
    if model.producer_name in ("pytorch", "tf2onnx"):
        return neural.NeuralNetwork.from_onnx(model)
    ops = [n.op_type for n in model.graph.node]
    found = [o for o in ops if o in _SUPPORTED]
    if len(found) > 1:
        raise ValueError("Incompatible ONNX graph provided: graph must contain at most one "
                         f"predictor operator, found {found}")
    if found:
        return _SUPPORTED[found[0]].from_onnx(model)
    n_weight_mats = sum(1 for t in model.graph.initializer if "coefficient" in t.name)
    if n_weight_mats > 1:
        if "ZipMap" in ops:
            return neural.MLPClassifier.from_onnx(model)
        return neural.MLPRegressor.from_onnx(model)
    raise ValueError("Incompatible ONNX graph provided: graph must contain a LinearRegressor "
                     "or LinearClassifier or TreeEnsembleRegressor or TreeEnsembleClassifier "
                     f"node, found: {ops}")
