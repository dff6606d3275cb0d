"""ONNX lookup helpers under the reference's module name (``pymoose.predictors.
predictor_utils``), so existing predictor code keeps importing them."""
from __future__ import annotations

from moose_amd.models.predictors.base import DEFAULT_FIXED_DTYPE  # noqa: F401
from moose_amd.models.predictors.base import DEFAULT_FLOAT_DTYPE  # noqa: F401
from moose_amd.models.predictors.base import find_attribute as find_attribute_in_node  # noqa: F401


def find_input_shape(input_node):
    return input_node.type.tensor_type.shape.dim


def find_node_in_model_proto(model_proto, operator_name, enforce=True):
    found = None
    for node in model_proto.graph.node:
        if node.name == operator_name or node.op_type == operator_name:
            found = node
    if enforce and found is None:
        raise ValueError(f"Model proto does not contain operator {operator_name}.")
    return found


def find_initializer_in_model_proto(model_proto, name, enforce=True):
    found = next((t for t in model_proto.graph.initializer if t.name == name), None)
    if enforce and found is None:
        raise ValueError(f"Model proto does not contain initializer {name}.")
    return found, (found.dims if found is not None else None)


def find_activation_in_model_proto(model_proto, output_name, enforce=True):
    found = next((n.name for n in model_proto.graph.node if n.output and n.output[0] == output_name),
                 None)
    if enforce and found is None:
        raise ValueError(f"Model proto does not produce {output_name}.")
    return found


def find_parameters_in_model_proto(model_proto, names, enforce=True):
    if isinstance(names, str):
        names = [names]
    params = [t for t in model_proto.graph.initializer if any(n in t.name for n in names)]
    if enforce and not params:
        raise ValueError(f"Model proto does not contain parameters matching {names}.")
    return params


def find_op_types_in_model_proto(model_proto, enforce=True):
    ops = [n.op_type for n in model_proto.graph.node]
    if enforce and not ops:
        raise ValueError("Model proto nodes do not contain op_type.")
    return ops


def find_output_in_model_proto(model_proto, enforce=True):
    out = model_proto.graph.output
    dims = out[0].type.tensor_type.shape.dim if out else None
    if enforce and dims is None:
        raise ValueError("Model proto does not contain an output dimension.")
    return dims
