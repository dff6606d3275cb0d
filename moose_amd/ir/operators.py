"""Operator catalogue of the native IR.

Parity: reference ``moose/src/computation.rs:828-914`` -- the 81 operators and their
attribute fields (``:922-1547``).  Each entry maps an operator name to its ordered
attribute schema ``[(attr, kind)]`` where ``kind`` drives both the textual parser and
the printer:

* ``int`` / ``opt_int`` / ``ints`` (list) / ``bool`` / ``str`` / ``key`` (16 raw bytes
  printed as hex) / ``const`` (a :class:`Constant`) / ``slice``.

Operators listed in ``EXTENSION_OPERATORS`` are this framework's fused host kernels
(one HIP launch for a whole RSS local step); they only appear in lowered graphs
produced by our compiler and are documented in ``docs/ARCHITECTURE.md``.
"""

OPERATORS = {
    "Abs": [],
    "Add": [],
    "And": [],
    "AtLeast2D": [("to_column_vector", "bool")],
    "BitExtract": [("bit_idx", "int")],
    "Broadcast": [("shape", "opt_ints")],
    "Cast": [],
    "Concat": [("axis", "int")],
    "Constant": [("value", "const")],
    "Decrypt": [],
    "DeriveSeed": [("sync_key", "key")],
    "Div": [],
    "Diag": [],
    "Dot": [],
    "ExpandDims": [("axis", "ints")],
    "Identity": [],
    "IndexAxis": [("axis", "int"), ("index", "int")],
    "Inverse": [],
    "Input": [("arg_name", "str")],
    "Load": [],
    "Mul": [],
    "Mean": [("axis", "opt_int")],
    "Output": [("tag", "str")],
    "Ones": [],
    "Or": [],
    "PrfKeyGen": [],
    "Reshape": [("shape", "opt_ints")],
    "Receive": [("rendezvous_key", "key"), ("sender", "str")],
    "Relu": [],
    "RingFixedpointArgmax": [("axis", "int"), ("upmost_index", "int")],
    "RingFixedpointDecode": [("scaling_base", "int"), ("scaling_exp", "int")],
    "RingFixedpointEncode": [("scaling_base", "int"), ("scaling_exp", "int")],
    "RingInject": [("bit_idx", "int")],
    "RingFixedpointMean": [
        ("axis", "opt_int"),
        ("scaling_base", "int"),
        ("scaling_exp", "int"),
    ],
    "Sample": [("max_value", "opt_int")],
    "SampleSeeded": [("max_value", "opt_int")],
    "Select": [("axis", "int")],
    "Send": [("rendezvous_key", "key"), ("receiver", "str")],
    "Save": [],
    "Shape": [],
    "Shl": [("amount", "int")],
    "Shr": [("amount", "int")],
    "Sign": [],
    "Slice": [("slice", "slice")],
    "Sqrt": [],
    "Squeeze": [("axis", "opt_int")],
    "Sub": [],
    "Sum": [("axis", "opt_int")],
    "Transpose": [],
    "Xor": [],
    "Zeros": [],
    "Equal": [],
    "EqualZero": [],
    "Exp": [],
    "FixedpointEncode": [("fractional_precision", "int"), ("integral_precision", "int")],
    "FixedpointDecode": [("fractional_precision", "int")],
    "Greater": [],
    "Less": [],
    "Neg": [],
    "Pow2": [],
    "Sigmoid": [],
    "AdtToRep": [],
    "AddN": [],
    "Argmax": [("axis", "int"), ("upmost_index", "int")],
    "BitDecompose": [],
    "BitCompose": [],
    "Fill": [("value", "const")],
    "Index": [("index", "int")],
    "Log2": [],
    "Log": [],
    "Maximum": [],
    "Msb": [],
    "Mux": [],
    "RepToAdt": [],
    "Reveal": [],
    "Share": [],
    "Softmax": [("axis", "int"), ("upmost_index", "int")],
    "ShlDim": [("amount", "int"), ("bit_length", "int")],
    "TruncPr": [("amount", "int")],
    "Demirror": [],
    "Mirror": [],
}

# Fused host kernels introduced by this framework's lowering (MI355X-first: one
# kernel per RSS local step instead of several tiny host ops).
EXTENSION_OPERATORS = {
    # z = x0*y0 + x0*y1 + x1*y0  (RSS multiplication cross terms)
    "RingMulCross": [],
    # z = x0.(y0+y1) + x1.y0     (RSS matmul cross terms, one K-concatenated GEMM)
    "RingDotCross": [],
    # z = x0&y0 ^ x0&y1 ^ x1&y0  (RSS AND cross terms on packed bit words)
    "BitAndCross": [],
    # zero share alpha_i = PRF(k_i) - PRF(k_{i+1}) expanded from two seeds
    "ZeroShare": [("bits", "int")],
    # logical right shift of a packed boolean word tensor along the bit axis
    "ShrWord": [("amount", "int")],
    "ShlWord": [("amount", "int")],
    # host primitives of lowered graphs that the reference expresses with other ops
    "Sar": [("amount", "int")],                      # arithmetic right shift
    "AddConst": [("value", "const")],                # x + public ring constant
    "RingCast": [],                                  # Z_2^128 -> Z_2^64 (width = ret type)
    "FromBool": [],
    "ToBool": [],
    "RingToInt": [],
    "IntToRing": [],
    "BitSplit": [("start", "int"), ("count", "int")],  # packed word -> bit planes
    "WeightedSum": [("weights", "ints"), ("bits", "int")],
    "StridedSlice": [("slices", "ints")],
    "MulLeading": [],  # x[i, ...] * c[i]: rank-agnostic public scaling (polymorphic plans)
}

ALL_OPERATORS = {**OPERATORS, **EXTENSION_OPERATORS}

# Deprecated operator names accepted by the parser (computation.rs:815-820).
OPERATOR_ALIASES = {
    "PrimDeriveSeed": "DeriveSeed",
    "PrimPrfKeyGen": "PrfKeyGen",
    "HostMean": "Mean",
    "FixedpointMeanOp": "Mean",
    "FloatingpointMeanOp": "Mean",
    "RepFixedpointMean": "Mean",
}

# Signature used when the textual form omits one (parsing.rs DeriveSeed).
DEFAULT_RETURN = {"DeriveSeed": "HostSeed", "PrfKeyGen": "HostPrfKey"}

assert len(OPERATORS) == 81, len(OPERATORS)
