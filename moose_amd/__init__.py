"""moose_amd -- an MI355X-native secure multi-party computation dataflow framework.

Drop-in for the ``pymoose`` API (reference ``pymoose/pymoose/__init__.py``)::

    import moose_amd as pm

    alice = pm.host_placement("alice")
    ...
    @pm.computation
    def f(x: pm.Argument(placement=alice, vtype=pm.TensorType(pm.float64))): ...

    pm.LocalMooseRuntime(["alice", "bob", "carole"]).set_default()
"""
from moose_amd.computation.dtypes import bool_  # noqa: F401
from moose_amd.computation.dtypes import fixed  # noqa: F401
from moose_amd.computation.dtypes import float32  # noqa: F401
from moose_amd.computation.dtypes import float64  # noqa: F401
from moose_amd.computation.dtypes import int32  # noqa: F401
from moose_amd.computation.dtypes import int64  # noqa: F401
from moose_amd.computation.dtypes import ring64  # noqa: F401
from moose_amd.computation.dtypes import uint32  # noqa: F401
from moose_amd.computation.dtypes import uint64  # noqa: F401
from moose_amd.computation.types import AesKeyType  # noqa: F401
from moose_amd.computation.types import AesTensorType  # noqa: F401
from moose_amd.computation.types import BytesType  # noqa: F401
from moose_amd.computation.types import FloatType  # noqa: F401
from moose_amd.computation.types import IntType  # noqa: F401
from moose_amd.computation.types import ShapeType  # noqa: F401
from moose_amd.computation.types import StringType  # noqa: F401
from moose_amd.computation.types import TensorType  # noqa: F401
from moose_amd.computation.types import UnitType  # noqa: F401
from moose_amd.edsl.base import Argument  # noqa: F401
from moose_amd.edsl.base import abs  # noqa: F401,A004
from moose_amd.edsl.base import add  # noqa: F401
from moose_amd.edsl.base import add_n  # noqa: F401
from moose_amd.edsl.base import argmax  # noqa: F401
from moose_amd.edsl.base import atleast_2d  # noqa: F401
from moose_amd.edsl.base import cast  # noqa: F401
from moose_amd.edsl.base import computation  # noqa: F401
from moose_amd.edsl.base import concatenate  # noqa: F401
from moose_amd.edsl.base import constant  # noqa: F401
from moose_amd.edsl.base import decrypt  # noqa: F401
from moose_amd.edsl.base import div  # noqa: F401
from moose_amd.edsl.base import dot  # noqa: F401
from moose_amd.edsl.base import exp  # noqa: F401
from moose_amd.edsl.base import expand_dims  # noqa: F401
from moose_amd.edsl.base import get_current_placement  # noqa: F401
from moose_amd.edsl.base import get_current_runtime  # noqa: F401
from moose_amd.edsl.base import greater  # noqa: F401
from moose_amd.edsl.base import host_placement  # noqa: F401
from moose_amd.edsl.base import identity  # noqa: F401
from moose_amd.edsl.base import index_axis  # noqa: F401
from moose_amd.edsl.base import inverse  # noqa: F401
from moose_amd.edsl.base import less  # noqa: F401
from moose_amd.edsl.base import load  # noqa: F401
from moose_amd.edsl.base import log  # noqa: F401
from moose_amd.edsl.base import log2  # noqa: F401
from moose_amd.edsl.base import logical_and  # noqa: F401
from moose_amd.edsl.base import logical_or  # noqa: F401
from moose_amd.edsl.base import maximum  # noqa: F401
from moose_amd.edsl.base import mean  # noqa: F401
from moose_amd.edsl.base import mirrored_placement  # noqa: F401
from moose_amd.edsl.base import mul  # noqa: F401
from moose_amd.edsl.base import mux  # noqa: F401
from moose_amd.edsl.base import ones  # noqa: F401
from moose_amd.edsl.base import output  # noqa: F401
from moose_amd.edsl.base import relu  # noqa: F401
from moose_amd.edsl.base import replicated_placement  # noqa: F401
from moose_amd.edsl.base import reshape  # noqa: F401
from moose_amd.edsl.base import save  # noqa: F401
from moose_amd.edsl.base import select  # noqa: F401
from moose_amd.edsl.base import set_current_runtime  # noqa: F401
from moose_amd.edsl.base import shape  # noqa: F401
from moose_amd.edsl.base import sigmoid  # noqa: F401
from moose_amd.edsl.base import sliced  # noqa: F401
from moose_amd.edsl.base import softmax  # noqa: F401
from moose_amd.edsl.base import sqrt  # noqa: F401
from moose_amd.edsl.base import square  # noqa: F401
from moose_amd.edsl.base import squeeze  # noqa: F401
from moose_amd.edsl.base import strided_slice  # noqa: F401
from moose_amd.edsl.base import sub  # noqa: F401
from moose_amd.edsl.base import sum  # noqa: F401,A004
from moose_amd.edsl.base import transpose  # noqa: F401
from moose_amd.edsl.base import zeros  # noqa: F401
from moose_amd.edsl.tracer import trace  # noqa: F401
from moose_amd.edsl.tracer import trace_and_compile  # noqa: F401
from moose_amd.runtime.local import LocalMooseRuntime  # noqa: F401


def __getattr__(name):
    # lazily imported heavier components
    if name == "GrpcMooseRuntime":
        from moose_amd.runtime.distributed import GrpcMooseRuntime

        return GrpcMooseRuntime
    if name == "DistributedMooseRuntime":
        from moose_amd.runtime.distributed import DistributedMooseRuntime

        return DistributedMooseRuntime
    if name == "MooseComputation":
        from moose_amd.compiler.api import MooseComputation

        return MooseComputation
    if name == "elk_compiler":
        import importlib

        return importlib.import_module("moose_amd.elk_compiler")
    if name == "predictors":
        from moose_amd.models import predictors

        return predictors
    raise AttributeError(name)


__version__ = "0.1.0"
