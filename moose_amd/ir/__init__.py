"""Native IR of moose_amd (types, operators, computations, textual + msgpack serde)."""
from moose_amd.ir.computation import AdditivePlacement  # noqa: F401
from moose_amd.ir.computation import Computation  # noqa: F401
from moose_amd.ir.computation import Constant  # noqa: F401
from moose_amd.ir.computation import HostPlacement  # noqa: F401
from moose_amd.ir.computation import Mirrored3Placement  # noqa: F401
from moose_amd.ir.computation import Operation  # noqa: F401
from moose_amd.ir.computation import ReplicatedPlacement  # noqa: F401
from moose_amd.ir.computation import SessionId  # noqa: F401
from moose_amd.ir.computation import Signature  # noqa: F401
from moose_amd.ir.types import TensorDType  # noqa: F401
from moose_amd.ir.types import Ty  # noqa: F401
