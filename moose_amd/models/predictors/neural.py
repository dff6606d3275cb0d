"""Dense neural networks: sklearn MLPs and PyTorch/Keras feed-forward nets.

Parity: reference ``pymoose/pymoose/predictors/multilayer_perceptron_predictor.py`` and
``neural_network_predictor.py``.  Each layer is one public-weight matmul (local on the
replicated placement + one truncation) and a public bias add; activations run inside
the MPC (ReLU = one comparison + mux, sigmoid/softmax via the fixed-point exp and
reciprocal protocols).

The ONNX import walks the graph instead of relying on initializer naming: ``Gemm``
(with ``transB``/``alpha``/``beta``) and ``MatMul`` + ``Add`` nodes with initializer
operands define layers, and activation nodes attach to the preceding layer.
"""
from __future__ import annotations

from enum import Enum
from typing import List
from typing import Optional

import numpy as np

import moose_amd as pm
from moose_amd.models.predictors.base import DEFAULT_FIXED_DTYPE
from moose_amd.models.predictors.base import Predictor
from moose_amd.models.predictors.base import find_attribute
from moose_amd.models.predictors.base import initializers
from moose_amd.models.predictors.base import load_onnx
from moose_amd.models.predictors.base import n_input_features


class Activation(Enum):
    IDENTITY = 1
    SIGMOID = 2
    SOFTMAX = 3
    RELU = 4


_ACT = {"Sigmoid": Activation.SIGMOID, "Relu": Activation.RELU, "Softmax": Activation.SOFTMAX}


def dense_layers_from_onnx(model):
    """-> (weights [in, out] list, biases list, activation per layer)."""
    init = initializers(model)
    ws: List[np.ndarray] = []
    bs: List[Optional[np.ndarray]] = []
    acts: List[Activation] = []
    for node in model.graph.node:
        op = node.op_type
        if op == "Gemm" and len(node.input) >= 2 and node.input[1] in init:
            w = init[node.input[1]]
            tb = find_attribute(node, "transB", enforce=False)
            if tb is not None and tb.i:
                w = w.T
            alpha = find_attribute(node, "alpha", enforce=False)
            if alpha is not None and alpha.f not in (0.0, 1.0):
                w = w * alpha.f
            b = init.get(node.input[2]) if len(node.input) > 2 else None
            beta = find_attribute(node, "beta", enforce=False)
            if b is not None and beta is not None and beta.f not in (0.0, 1.0):
                b = b * beta.f
            ws.append(w)
            bs.append(None if b is None else b.reshape(-1))
            acts.append(Activation.IDENTITY)
        elif op == "MatMul" and node.input[1] in init:
            ws.append(init[node.input[1]])
            bs.append(None)
            acts.append(Activation.IDENTITY)
        elif op == "Add" and ws and bs[-1] is None and any(i in init for i in node.input):
            b = init[next(i for i in node.input if i in init)]
            bs[-1] = b.reshape(-1)
        elif op in _ACT and ws:
            acts[-1] = _ACT[op]
    if not ws:
        raise ValueError("no dense layers found in the ONNX graph")
    bs = [b if b is not None else np.zeros(w.shape[1]) for w, b in zip(ws, bs)]
    nf = n_input_features(model)
    if ws[0].shape[0] != nf:
        raise ValueError(f"the model input has {nf} features but the first layer's weights "
                         f"have shape {ws[0].shape}")
    return ws, bs, acts


class DenseNetwork(Predictor):
    def __init__(self, weights, biases, activations):
        super().__init__()
        self.weights = [np.asarray(w, dtype=np.float64) for w in weights]
        self.biases = [np.asarray(b, dtype=np.float64).reshape(-1) for b in biases]
        self.activations = list(activations)
        for w, b in zip(self.weights, self.biases):
            if w.shape[1] != b.shape[0]:
                raise ValueError(f"layer weight {w.shape} and bias {b.shape} mismatch")

    @property
    def n_outputs(self):
        return self.biases[-1].shape[0]

    def layer(self, x, i, fixedpoint_dtype):
        w = self.fixedpoint_constant(self.weights[i], plc=self.mirrored, dtype=fixedpoint_dtype)
        b = self.fixedpoint_constant(self.biases[i], plc=self.mirrored, dtype=fixedpoint_dtype)
        return pm.add(pm.dot(x, w), b)

    def activate(self, z, act: Activation):
        if act is Activation.SIGMOID:
            return pm.sigmoid(z)
        if act is Activation.RELU:
            return pm.relu(z)
        if act is Activation.SOFTMAX:
            return pm.softmax(z, axis=1, upmost_index=self.n_outputs)
        return z

    def forward(self, x, fixedpoint_dtype, acts):
        for i in range(len(self.weights)):
            x = self.activate(self.layer(x, i, fixedpoint_dtype), acts[i])
        return x


class NeuralNetwork(DenseNetwork):
    """Feed-forward network exported from PyTorch (``Gemm``) or Keras/tf2onnx
    (``MatMul`` + ``Add``); activations as found in the graph."""

    def predict(self, x, fixedpoint_dtype=DEFAULT_FIXED_DTYPE):
        return self.forward(x, fixedpoint_dtype, self.activations)

    @classmethod
    def from_onnx(cls, model):
        return cls(*dense_layers_from_onnx(load_onnx(model)))


class MLPPredictor(DenseNetwork):
    """sklearn MLP: one hidden activation for every hidden layer, none on the output
    layer, then the estimator-specific post transform."""

    def __init__(self, weights, biases, activation=Activation.IDENTITY):
        n = len(weights)
        super().__init__(weights, biases, [activation] * (n - 1) + [Activation.IDENTITY])
        self.activation = activation

    def post_transform(self, y, fixedpoint_dtype):
        return y

    def predict(self, x, fixedpoint_dtype=DEFAULT_FIXED_DTYPE):
        return self.post_transform(self.forward(x, fixedpoint_dtype, self.activations),
                                   fixedpoint_dtype)

    @classmethod
    def from_onnx(cls, model):
        ws, bs, acts = dense_layers_from_onnx(load_onnx(model))
        hidden = acts[0] if len(acts) > 1 else Activation.IDENTITY
        if hidden is Activation.SOFTMAX:
            hidden = Activation.IDENTITY
        return cls(ws, bs, hidden)


class MLPRegressor(MLPPredictor):
    pass


class MLPClassifier(MLPPredictor):
    def post_transform(self, y, fixedpoint_dtype):
        if self.n_outputs == 1:  # binary: probabilities of both classes
            p = pm.sigmoid(y)
            one = self.fixedpoint_constant(1.0, plc=self.mirrored, dtype=fixedpoint_dtype)
            return pm.concatenate([pm.sub(one, p), p], axis=1)
        return pm.softmax(y, axis=1, upmost_index=self.n_outputs)
