"""Linear models: regression and (logistic) classification.

Parity: reference ``pymoose/pymoose/predictors/linear_predictor.py``.  One secure
matmul with public (mirrored) weights -- a local GEMM on the replicated placement
followed by one truncation -- plus a public bias add; classifiers then apply the
post-transform (sigmoid, normalised sigmoid or softmax) inside the MPC.
"""
from __future__ import annotations

from enum import Enum

import numpy as np

import moose_amd as pm
from moose_amd.models.predictors.base import DEFAULT_FIXED_DTYPE
from moose_amd.models.predictors.base import Predictor
from moose_amd.models.predictors.base import find_attribute
from moose_amd.models.predictors.base import find_node
from moose_amd.models.predictors.base import load_onnx
from moose_amd.models.predictors.base import n_input_features
from moose_amd.models.predictors.onnx_proto import FLOATS


class PostTransform(Enum):
    NONE = 1
    SIGMOID = 2
    SOFTMAX = 3


def _as_matrix(coeffs):
    c = np.asarray(coeffs, dtype=np.float64)
    if c.ndim == 1:
        c = c[None, :]
    if c.ndim != 2:
        raise ValueError(f"coefficients must be rank 1 or 2, got shape {c.shape}")
    return c


def _as_vector(b, n):
    if b is None:
        return None
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    if b.shape[0] != n:
        raise ValueError(f"{b.shape[0]} intercepts for {n} outputs")
    return b


class LinearPredictor(Predictor):
    def __init__(self, coeffs, intercepts=None):
        super().__init__()
        self.coeffs = _as_matrix(coeffs)  # [n_outputs, n_features]
        self.intercepts = _as_vector(intercepts, self.coeffs.shape[0])

    def linear(self, x, fixedpoint_dtype):
        w = self.fixedpoint_constant(self.coeffs.T, plc=self.mirrored, dtype=fixedpoint_dtype)
        y = pm.dot(x, w)
        if self.intercepts is not None:
            b = self.fixedpoint_constant(self.intercepts, plc=self.mirrored, dtype=fixedpoint_dtype)
            y = pm.add(y, b)
        return y

    def post_transform(self, y):
        return y

    def predict(self, x, fixedpoint_dtype=DEFAULT_FIXED_DTYPE):
        return self.post_transform(self.linear(x, fixedpoint_dtype))

    @staticmethod
    def _floats(node, name, enforce=True):
        a = find_attribute(node, name, enforce)
        if a is None:
            return None
        if a.type != FLOATS:
            raise ValueError(f"{node.op_type} {name} must be of type FLOATS")
        return np.asarray(a.floats, dtype=np.float64)


class LinearRegressor(LinearPredictor):
    @classmethod
    def from_onnx(cls, model):
        model = load_onnx(model)
        node = find_node(model, "LinearRegressor", enforce=False)
        if node is None:
            raise ValueError("Incompatible ONNX graph provided: graph must contain a "
                             "LinearRegressor operator.")
        coeffs = cls._floats(node, "coefficients")
        intercepts = cls._floats(node, "intercepts", enforce=False)
        targets = find_attribute(node, "targets", enforce=False)
        coeffs = coeffs.reshape(int(targets.i) if targets is not None else 1, -1)
        nf = n_input_features(model)
        if coeffs.shape[1] != nf:
            raise ValueError(f"the model input has {nf} features but there are "
                             f"{coeffs.shape[1]} coefficients per target")
        return cls(coeffs, intercepts)


class LinearClassifier(LinearPredictor):
    def __init__(self, coeffs, intercepts=None, post_transform=PostTransform.NONE):
        super().__init__(coeffs, intercepts)
        self.n_classes = self.coeffs.shape[0]
        if not isinstance(post_transform, PostTransform):
            raise ValueError("Could not infer post-transform in LinearClassifier")
        self.transform = post_transform

    def post_transform(self, y):
        if self.transform is PostTransform.NONE:
            return y
        if self.transform is PostTransform.SOFTMAX:
            return pm.softmax(y, axis=1, upmost_index=self.n_classes)
        s = pm.sigmoid(y)
        if self.n_classes == 2:
            return s
        # one-vs-rest sigmoid scores normalised to sum to one (sklearn "ovr")
        return pm.div(s, pm.expand_dims(pm.sum(s, axis=1), 1))

    @classmethod
    def from_onnx(cls, model):
        model = load_onnx(model)
        node = find_node(model, "LinearClassifier", enforce=False)
        if node is None:
            raise ValueError("Incompatible ONNX graph provided: graph must contain a "
                             "LinearClassifier operator.")
        coeffs = cls._floats(node, "coefficients")
        labels = (find_attribute(node, "classlabels_ints", enforce=False)
                  or find_attribute(node, "classlabels_strings", enforce=False))
        if labels is None:
            raise ValueError("LinearClassifier without class labels")
        n_classes = len(labels.ints) or len(labels.strings)
        coeffs = coeffs.reshape(n_classes, -1)
        nf = n_input_features(model)
        if coeffs.shape[1] != nf:
            raise ValueError(f"the model input has {nf} features but there are "
                             f"{coeffs.shape[1]} coefficients per class")
        intercepts = cls._floats(node, "intercepts", enforce=False)
        pt = find_attribute(node, "post_transform").s.decode()
        transforms = {"NONE": PostTransform.NONE, "LOGISTIC": PostTransform.SIGMOID,
                      "SOFTMAX": PostTransform.SOFTMAX}
        if pt not in transforms:
            raise RuntimeError(f"{pt} post_transform is unsupported for LinearClassifier.")
        return cls(coeffs, intercepts, transforms[pt])
