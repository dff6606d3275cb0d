"""Trace an :class:`AbstractComputation` into an eDSL :class:`Computation`.

Parity: reference ``pymoose/pymoose/edsl/tracer.py:13-64`` (trace / auto-Output /
role_map).  Instead of one ``visit_*`` method per expression class, one table maps
each expression ``kind`` to (operation class, operand names, name prefix).
"""
import inspect
from collections import defaultdict

from moose_amd.computation import computation as comp
from moose_amd.computation import operations as ops
from moose_amd.computation import placements as plc
from moose_amd.computation import types as ty
from moose_amd.edsl import base as expr

# kind -> (Operation class name, operand names or "array"/"unary", fresh-name prefix,
#          attribute names copied from expression attrs)
_OPS = {
    "identity": ("IdentityOperation", ["x"], "identity", []),
    "add_n": ("AddNOperation", "array", "add_n", []),
    "concatenate": ("ConcatenateOperation", "array", "concatenate", ["axis"]),
    "maximum": ("MaximumOperation", "array", "maximum", []),
    "decrypt": ("DecryptOperation", ["key", "ciphertext"], "decrypt", []),
    "constant": ("ConstantOperation", [], "constant", ["value"]),
    "add": ("AddOperation", ["lhs", "rhs"], "add", []),
    "sub": ("SubOperation", ["lhs", "rhs"], "sub", []),
    "mul": ("MulOperation", ["lhs", "rhs"], "mul", []),
    "div": ("DivOperation", ["lhs", "rhs"], "div", []),
    "dot": ("DotOperation", ["lhs", "rhs"], "dot", []),
    "and": ("BitwiseAndOperation", ["lhs", "rhs"], "and", []),
    "or": ("BitwiseOrOperation", ["lhs", "rhs"], "or", []),
    "less": ("LessOperation", ["lhs", "rhs"], "less", []),
    "greater": ("GreaterOperation", ["lhs", "rhs"], "greater", []),
    "inverse": ("InverseOperation", ["x"], "inverse", []),
    "abs": ("AbsOperation", ["x"], "abs", []),
    "cast": ("CastOperation", ["x"], "cast", []),
    "expand_dims": ("ExpandDimsOperation", ["x"], "expand_dims", ["axis"]),
    "exp": ("ExpOperation", ["x"], "exp", []),
    "sqrt": ("SqrtOperation", ["x"], "sqrt", []),
    "sigmoid": ("SigmoidOperation", ["x"], "sigmoid", []),
    "relu": ("ReluOperation", ["x"], "relu", []),
    "log": ("LogOperation", ["x"], "log", []),
    "log2": ("Log2Operation", ["x"], "log2", []),
    "softmax": ("SoftmaxOperation", ["x"], "softmax", ["axis", "upmost_index"]),
    "argmax": ("ArgmaxOperation", ["x"], "argmax", ["axis", "upmost_index"]),
    "squeeze": ("SqueezeOperation", ["x"], "squeeze", ["axis"]),
    "ones": ("OnesOperation", ["shape"], "ones", []),
    "zeros": ("ZerosOperation", ["shape"], "zeros", []),
    "sum": ("SumOperation", ["x"], "sum", ["axis"]),
    "mean": ("MeanOperation", ["x"], "mean", ["axis"]),
    "transpose": ("TransposeOperation", ["x"], "transpose", []),
    "reshape": ("ReshapeOperation", ["x", "shape"], "reshape", []),
    "atleast_2d": ("AtLeast2DOperation", ["x"], "atleast_2d", ["to_column_vector"]),
    "index_axis": ("IndexAxisOperation", ["x"], "index_axis", ["axis", "index"]),
    "select": ("SelectOperation", ["x", "index"], "select", ["axis"]),
    "slice": ("SliceOperation", ["x"], "slice", ["begin", "end"]),
    "strided_slice": ("StridedSliceOperation", ["x"], "strided_slice", ["slices"]),
    "shape": ("ShapeOperation", ["x"], "shape", []),
    "mux": ("MuxOperation", ["selector", "x", "y"], "mux", []),
    "load": ("LoadOperation", ["key", "query"], "load", []),
    "save": ("SaveOperation", ["key", "value"], "save", []),
    "output": ("OutputOperation", ["value"], "output", ["tag"]),
}


def _resolve_annotation(func, ann):
    """Evaluate string annotations (``from __future__ import annotations``) in the
    function's globals plus its closure."""
    if not isinstance(ann, str):
        return ann
    scope = dict(func.__globals__)
    if func.__closure__:
        for name, cell in zip(func.__code__.co_freevars, func.__closure__):
            try:
                scope[name] = cell.cell_contents
            except ValueError:
                pass
    return eval(ann, scope)  # noqa: S307 - annotations are user code


def trace(abstract_computation):
    func = abstract_computation.func
    params = inspect.signature(func).parameters
    symbolic_args = []
    for arg_name, p in params.items():
        ann = _resolve_annotation(func, p.annotation)
        if not isinstance(ann, expr.Argument):
            raise TypeError(f"Parameter `{arg_name}` must be annotated with pm.Argument")
        symbolic_args.append(
            expr.Expression("argument", ann.placement, [], ann.vtype, {"arg_name": arg_name})
        )
    result = abstract_computation.func(*symbolic_args)
    return AstTracer(role_map=abstract_computation.role_map).trace(result)


def trace_and_compile(abstract_computation, compiler_passes=None):
    from moose_amd import elk_compiler

    logical = trace(abstract_computation)
    return elk_compiler.compile_computation(logical, compiler_passes)


class AstTracer:
    def __init__(self, role_map=None):
        self.computation = comp.Computation(operations={}, placements={})
        self.name_counters = defaultdict(int)
        self.operation_cache = {}
        self.placement_cache = {}
        self.role_map = role_map

    def get_fresh_name(self, prefix):
        n = self.name_counters[prefix]
        self.name_counters[prefix] += 1
        return f"{prefix}_{n}"

    def trace(self, expressions):
        if not isinstance(expressions, (tuple, list)):
            expressions = [expressions]
        for e in expressions:
            op = self.visit(e)
            if not isinstance(op, ops.OutputOperation):
                name = self.get_fresh_name("output")
                self.computation.add_operation(
                    ops.OutputOperation(
                        name=name,
                        inputs={"value": op.name},
                        placement_name=op.placement_name,
                        signature=ops.OpSignature(
                            input_types={"value": op.return_type},
                            return_type=op.return_type,
                        ),
                        tag=name,
                    )
                )
        return self.computation

    # placements ------------------------------------------------------------
    def visit_placement_expression(self, p):
        if p in self.placement_cache:
            return self.placement_cache[p]
        if isinstance(p, expr.HostPlacementExpression):
            placement = plc.HostPlacement(name=self._role(p.name))
        elif isinstance(p, (expr.ReplicatedPlacementExpression, expr.MirroredPlacementExpression)):
            players = [self.visit_placement_expression(q).name for q in p.players]
            cls = (
                plc.ReplicatedPlacement
                if isinstance(p, expr.ReplicatedPlacementExpression)
                else plc.MirroredPlacement
            )
            placement = cls(name=self._role(p.name), player_names=players)
        else:
            raise TypeError(f"Unknown placement expression {type(p)}")
        placement = self.computation.maybe_add_placement(placement)
        self.placement_cache[p] = placement
        return placement

    def _role(self, name):
        if self.role_map is None:
            return name
        swapped = self.role_map.get(name, name)
        # role maps may use placement expressions as keys/values
        if isinstance(swapped, expr.PlacementExpression):
            swapped = swapped.name
        for k, v in self.role_map.items():
            if isinstance(k, expr.PlacementExpression) and k.name == name:
                swapped = v.name if isinstance(v, expr.PlacementExpression) else v
        return swapped

    # expressions -------------------------------------------------------------
    def visit(self, e):
        if e not in self.operation_cache:
            self.operation_cache[e] = self._visit(e)
        return self.operation_cache[e]

    def _visit(self, e):
        if not isinstance(e, expr.Expression):
            raise TypeError(f"Cannot trace value of type {type(e)}")
        placement = self.visit_placement_expression(e.placement)
        if e.kind == "argument":
            return self.computation.add_operation(
                ops.InputOperation(
                    name=e.attrs["arg_name"],
                    inputs={},
                    placement_name=placement.name,
                    signature=ops.OpSignature({}, e.vtype or ty.UnknownType()),
                )
            )
        cls_name, operands, prefix, attr_names = _OPS[e.kind]
        input_ops = [self.visit(i) for i in e.inputs]
        if operands == "array":
            operands = [f"array{i}" for i in range(len(input_ops))]
        inputs = {n: op.name for n, op in zip(operands, input_ops)}
        input_types = {n: op.return_type for n, op in zip(operands, input_ops)}
        if e.kind == "save":
            return_type = ty.UnitType()
        elif e.kind == "output":
            return_type = input_ops[0].return_type
        else:
            return_type = e.vtype if e.vtype is not None else ty.UnknownType()
        attrs = {a: e.attrs.get(a) for a in attr_names}
        cls = ops.OPERATION_CLASSES[cls_name]
        return self.computation.add_operation(
            cls(
                name=self.get_fresh_name(prefix),
                inputs=inputs,
                placement_name=placement.name,
                signature=ops.OpSignature(input_types, return_type),
                **attrs,
            )
        )
