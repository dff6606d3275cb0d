"""Predictor base class, ONNX helpers and the AES input wrapper.

Parity: reference ``pymoose/pymoose/predictors/predictor.py`` (``Predictor``,
``AesWrapper``) and ``predictor_utils.py`` (ONNX lookups, default dtypes).  Model
parameters are public constants on the *mirrored* placement (so products with them are
local on the replicated placement), inputs are secret on the replicated placement, and
results are opened on a chosen host.
"""
from __future__ import annotations

import numpy as np

import moose_amd as pm
from moose_amd.models.predictors import onnx_proto

DEFAULT_FLOAT_DTYPE = pm.float64
DEFAULT_FIXED_DTYPE = pm.fixed(24, 40)


class Predictor:
    """Standard placements: hosts alice/bob/carole, their mirrored and replicated
    groupings."""

    def __init__(self):
        self.alice = pm.host_placement("alice")
        self.bob = pm.host_placement("bob")
        self.carole = pm.host_placement("carole")
        players = [self.alice, self.bob, self.carole]
        self.replicated = pm.replicated_placement(name="replicated", players=players)
        self.mirrored = pm.mirrored_placement(name="mirrored", players=players)

    @property
    def host_placements(self):
        return self.alice, self.bob, self.carole

    def predict(self, x, fixedpoint_dtype=DEFAULT_FIXED_DTYPE):  # pragma: no cover
        raise NotImplementedError

    def __call__(self, x, fixedpoint_dtype=DEFAULT_FIXED_DTYPE):
        return self.predict(x, fixedpoint_dtype)

    @classmethod
    def fixedpoint_constant(cls, x, plc=None, dtype=DEFAULT_FIXED_DTYPE):
        """A float constant embedded in the computation and cast to fixed point."""
        c = pm.constant(np.asarray(x, dtype=np.float64) if not np.isscalar(x) else float(x),
                        dtype=pm.float64, placement=plc)
        return pm.cast(c, dtype=dtype, placement=plc)

    @classmethod
    def handle_output(cls, prediction, prediction_handler, output_dtype=DEFAULT_FLOAT_DTYPE):
        with prediction_handler:
            return pm.cast(prediction, dtype=output_dtype)

    def predictor_factory(self, fixedpoint_dtype=DEFAULT_FIXED_DTYPE):
        """A ready-to-run computation: float input on alice, prediction opened on bob."""

        @pm.computation
        def predictor(x: pm.Argument(self.alice, dtype=pm.float64)):
            with self.alice:
                xf = pm.cast(x, dtype=fixedpoint_dtype)
            with self.replicated:
                y = self(xf, fixedpoint_dtype)
            return self.handle_output(y, prediction_handler=self.bob)

        return predictor


def AesWrapper(model_cls):  # noqa: N802 - reference API name
    """Extend a predictor class so its computation takes AES-encrypted inputs that are
    decrypted inside the replicated placement (reference predictor.py:49-85)."""

    class AesPredictor(model_cls):
        def __call__(self, fixedpoint_dtype=DEFAULT_FIXED_DTYPE):
            return self.aes_predictor_factory(fixedpoint_dtype)

        @classmethod
        def handle_aes_input(cls, aes_key, aes_data, decryptor):
            with decryptor:
                return pm.decrypt(aes_key, aes_data)

        def aes_predictor_factory(self, fixedpoint_dtype=DEFAULT_FIXED_DTYPE):
            @pm.computation
            def predictor(aes_data: pm.Argument(self.alice, vtype=pm.AesTensorType(
                    dtype=fixedpoint_dtype)),
                          aes_key: pm.Argument(self.replicated, vtype=pm.AesKeyType())):
                x = self.handle_aes_input(aes_key, aes_data, decryptor=self.replicated)
                with self.replicated:
                    y = self.predict(x, fixedpoint_dtype)
                return self.handle_output(y, prediction_handler=self.bob)

            return predictor

    AesPredictor.__name__ = f"Aes{model_cls.__name__}"
    return AesPredictor


# ---------------------------------------------------------------------------
# ONNX helpers (reference predictor_utils.py)
# ---------------------------------------------------------------------------
def load_onnx(model):
    """Accept a decoded ModelProto, a path, bytes or a file object."""
    if hasattr(model, "graph"):
        return model
    return onnx_proto.load_model(model)


def find_node(model, op_type, enforce=True):
    """First node whose op_type (or name, as the reference matches) is ``op_type``."""
    for n in model.graph.node:
        if n.op_type == op_type or n.name == op_type:
            return n
    if enforce:
        raise ValueError(f"Model proto does not contain operator {op_type}.")
    return None


def find_attribute(node, name, enforce=True):
    for a in node.attribute:
        if a.name == name:
            return a
    if enforce:
        raise ValueError(f"Node {node.name} does not contain attribute {name}.")
    return None


def n_input_features(model) -> int:
    dims = model.graph.input[0].type.tensor_type.shape.dim
    if len(dims) != 2:
        raise ValueError("predictors expect a rank-2 [batch, features] model input")
    return int(dims[1].dim_value)


def initializers(model):
    return {t.name: onnx_proto.to_array(t).astype(np.float64) for t in model.graph.initializer}
