"""Error model.

Parity: reference ``moose/src/error.rs:7-61`` -- one ``Error`` enum with 17 variants.
Here every variant is a subclass of :class:`MooseError`, and the subsystem errors raised
throughout the framework (interpreter, graph executor, compiler, transport, native
kernels, parser, distributed runtime) derive from the matching variant, so callers can
catch either the precise subsystem error or the reference's category.
"""
from __future__ import annotations


class MooseError(RuntimeError):
    """Base of every framework error."""


class Unexpected(MooseError):
    pass


class OperandUnavailable(MooseError):
    """A kernel operand never arrived (e.g. a Receive without its Send)."""


class ResultUnused(MooseError):
    pass


class TypeMismatch(MooseError):
    def __init__(self, expected, found):
        super().__init__(f"Type mismatch, expected {expected} but found {found}")
        self.expected, self.found = expected, found


class UnimplementedOperator(MooseError):
    pass


class KernelError(MooseError):
    """A native (HIP or host) kernel reported failure."""


class MissingArgument(MooseError):
    pass


class InvalidArgument(MooseError, ValueError):
    pass


class MalformedEnvironment(MooseError):
    """An operand name is not bound in the environment."""


class MalformedComputation(MooseError):
    pass


class MalformedPlacement(MooseError):
    pass


class Compilation(MooseError):
    pass


class Networking(MooseError):
    pass


class Storage(MooseError):
    pass


class TestRuntime(MooseError):
    __test__ = False  # not a pytest test class


class SessionAlreadyExists(MooseError):
    pass


class SerializationError(MooseError):
    pass


VARIANTS = (Unexpected, OperandUnavailable, ResultUnused, TypeMismatch, UnimplementedOperator,
            KernelError, MissingArgument, InvalidArgument, MalformedEnvironment,
            MalformedComputation, MalformedPlacement, Compilation, Networking, Storage,
            TestRuntime, SessionAlreadyExists, SerializationError)
