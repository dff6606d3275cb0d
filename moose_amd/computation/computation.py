"""Container for a traced eDSL computation (``pymoose.computation.computation``)."""
from dataclasses import dataclass
from dataclasses import field
from typing import Dict

from moose_amd.computation import operations as ops
from moose_amd.computation import placements as plc


@dataclass
class Computation:
    operations: Dict[str, ops.Operation] = field(default_factory=dict)
    placements: Dict[str, plc.Placement] = field(default_factory=dict)

    # lookups ---------------------------------------------------------------
    def operation(self, name):
        return self.operations[name]

    def placement(self, name):
        return self.placements[name]

    def find_operations_of_type(self, op_type):
        return [op for op in self.operations.values() if isinstance(op, op_type)]

    def find_destinations(self, op):
        return [c for c in self.operations.values() if op.name in c.inputs.values()]

    def find_sources(self, op):
        return [self.operation(n) for n in op.inputs.values()]

    # mutation --------------------------------------------------------------
    def add(self, component):
        if isinstance(component, ops.Operation):
            return self.add_operation(component)
        if isinstance(component, plc.Placement):
            return self.add_placement(component)
        raise NotImplementedError(f"{component}")

    def maybe_add(self, component):
        if isinstance(component, ops.Operation):
            return self.maybe_add_operation(component)
        if isinstance(component, plc.Placement):
            return self.maybe_add_placement(component)
        raise NotImplementedError(f"{component}")

    def add_placement(self, placement):
        assert isinstance(placement, plc.Placement)
        assert placement.name not in self.placements, placement.name
        self.placements[placement.name] = placement
        return placement

    def maybe_add_placement(self, placement):
        existing = self.placements.get(placement.name)
        if existing is not None:
            assert existing == placement, (existing, placement)
            return existing
        return self.add_placement(placement)

    def add_operation(self, op):
        assert isinstance(op, ops.Operation)
        assert op.name not in self.operations, op.name
        assert op.placement_name in self.placements, op.placement_name
        self.operations[op.name] = op
        return op

    def maybe_add_operation(self, op):
        existing = self.operations.get(op.name)
        if existing is not None:
            assert existing == op
            return existing
        return self.add_operation(op)

    def add_operations(self, operations):
        for op in operations:
            self.add_operation(op)

    def remove_operation(self, name):
        del self.operations[name]

    def remove_operations(self, names):
        for name in names:
            self.remove_operation(name)

    def rewire(self, old_op, new_op):
        assert old_op.name in self.operations and new_op.name in self.operations
        for op in self.operations.values():
            for k, v in op.inputs.items():
                if v == old_op.name:
                    op.inputs[k] = new_op.name
